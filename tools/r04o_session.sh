cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04o && mkdir -p $O
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) tools/host_overhead_probe.py > $O/probe.json 2> $O/probe.err || { echo failed; tail -30 $O/probe.err; exit 1; }
grep "^{" $O/probe.json
echo done
