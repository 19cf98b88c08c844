cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04m && mkdir -p $O
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --gather-obs --global-envs 32768 --steps 2000 --warmup 500 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 > $O/g1_delta.json 2> $O/g1_delta.err || { echo failed; tail $O/g1_delta.err; exit 1; }
python -c "import json; d=json.load(open('$O/g1_delta.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('gather'))[:500], json.dumps(d.get('no_gather'))[:300])"
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 1 --gather-obs --gather-mode full --global-envs 32768 --steps 2000 --warmup 500 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 > $O/g1_full.json 2> $O/g1_full.err || { echo failed; tail $O/g1_full.err; exit 1; }
python -c "import json; d=json.load(open('$O/g1_full.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('gather'))[:500])"
echo done
