cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04h && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 170 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d['delta_exchange'])); print(json.dumps(d['collect'])[:400])"
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof bench failed"; tail $O/prof_bench.err; exit 1; }
bash tools/pmc_valu.sh r04h/pmc 262144 || exit 1
echo done
