cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04p && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_bench_gpu.py tests/test_delta_gather_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) tools/host_overhead_probe.py > $O/probe.json 2> $O/probe.err || { echo failed; tail -30 $O/probe.err; exit 1; }
grep "^{" $O/probe.json
for gm in delta full; do
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 1 --gather-obs --gather-mode $gm --global-envs 32768 --steps 2000 --warmup 500 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --weak-envs 0 > $O/g1_$gm.json 2> $O/g1_$gm.err || { echo failed; tail $O/g1_$gm.err; exit 1; }
grep "^{" $O/g1_$gm.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$gm', d['value'], d['ms_per_step']*1e3, d['gather']['overflows'], d['no_gather']['ms_per_step']*1e3)"
done
echo done
