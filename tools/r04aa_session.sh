# native exchange in one call per env-step: GPU tests, the gather bench (native / torch), the host
# probe; then the PMC passes of this build and the default bench line with them
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04aa && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_delta_gather_gpu.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for ex in native torch; do
CF2SIM_EXCHANGE=$ex timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 1 --gather-obs --gather-mode delta --global-envs 32768 --steps 2000 --warmup 500 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --weak-envs 0 > $O/g1_$ex.json 2> $O/g1_$ex.err || { echo failed; tail $O/g1_$ex.err; exit 1; }
grep "^{" $O/g1_$ex.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ex', d['value'], d['ms_per_step']*1e3, d['gather']['exchange'], d['gather']['overflows'], d['no_gather']['ms_per_step']*1e3)"
done
CF2SIM_EXCHANGE=native timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) tools/host_overhead_probe.py > $O/probe.json 2> $O/probe.err || { echo probe failed; tail -30 $O/probe.err; exit 1; }
grep "^{" $O/probe.json
bash tools/pmc_traffic.sh r04aa/traffic 262144 || exit 1
cp $O/traffic/step_kernel_traffic.json profiles/step_kernel_traffic.json
bash tools/pmc_valu.sh r04aa/pmc 262144 || exit 1
bash tools/r04y_session.sh || exit 1
echo done
