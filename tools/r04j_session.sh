cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04j && mkdir -p $O
bash tools/pmc_traffic.sh r04j/traffic 262144 || exit 1
bash tools/all_configs.sh $O/all_configs.jsonl || { echo all_configs failed; exit 1; }
timeout -k 10 170 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['roofline'])[:600])"
echo done
