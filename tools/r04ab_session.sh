# the native exchange with the time-out count copies in the C call: GPU tests and the gather bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ab && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_delta_gather_gpu.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for ex in native torch native; do
CF2SIM_EXCHANGE=$ex timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 1 --gather-obs --gather-mode delta --global-envs 32768 --steps 2000 --warmup 500 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --weak-envs 0 > $O/g1_$ex.json 2> $O/g1_$ex.err || { echo failed; tail $O/g1_$ex.err; exit 1; }
grep "^{" $O/g1_$ex.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ex', d['value'], d['ms_per_step']*1e3, d['gather']['exchange'], d['gather']['overflows'], d['no_gather']['ms_per_step']*1e3)"
done
echo done
