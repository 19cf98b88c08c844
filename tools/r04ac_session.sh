# kernel trace of the delta-gather bench at the node shard (one RCCL rank, native exchange): where
# the GPU time of a step with its exchange goes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ac && mkdir -p $O
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 400))
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o g -- python3 bench.py --gpus 1 --gather-obs --gather-mode delta --global-envs 32768 --steps 2000 --warmup 500 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --weak-envs 0 > $O/g.json 2> $O/g.err || { echo failed; tail $O/g.err; exit 1; }
grep "^{" $O/g.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1e3, d['gather']['exchange'])"
head -12 $O/prof/g_kernel_stats.csv
python3 - $O/prof/g_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-400:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[-40:]:
    print(r["Kernel_Name"][:50], r.get("Queue_Id"), r.get("Stream_Id"), (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
PY
echo done
