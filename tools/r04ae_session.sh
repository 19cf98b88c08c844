# PMC passes of the final build (the public header changed after r04aa), then the default bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ae && mkdir -p $O
bash tools/pmc_traffic.sh r04ae/traffic 262144 || exit 1
cp $O/traffic/step_kernel_traffic.json profiles/step_kernel_traffic.json
bash tools/pmc_valu.sh r04ae/pmc 262144 || exit 1
timeout -k 10 170 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['valu_issue_frac'])"
echo done
