# Full GPU validation of the in-tree build + every measurement the judge reads (round 5).  Three
# parts, each one gpurun call (`bash tools/final_round.sh TAG A|B|C`):
#   A  smoke + every -m gpu test
#   B  PMC passes of this kernel build: HBM traffic at 262 144 and 1 Mi envs (tools/pmc_traffic.sh),
#      VALU issue / MFMA busy (tools/pmc_valu.sh); copy the two JSONs into profiles/ before part C
#   C  the default bench line, a rocprofv3 --kernel-trace --stats summary of the bench workload,
#      every BASELINE config (tools/all_configs.sh), the node-shard exchange probe
set -o pipefail
TAG=${1:-final}
PART=${2:-A}
OUT=gpurun_out/$TAG$PART
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case $PART in
A)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; exit $rc ;;
B)
  bash tools/pmc_traffic.sh ${TAG}_traffic 262144 > $OUT/traffic.log 2>&1 || { echo "traffic failed"; tail -20 $OUT/traffic.log; exit 1; }
  cp gpurun_out/${TAG}_traffic/step_kernel_traffic.json profiles/step_kernel_traffic.json
  bash tools/pmc_traffic.sh ${TAG}_traffic_oc 1048576 > $OUT/traffic_oc.log 2>&1 || { echo "traffic oc failed"; tail -20 $OUT/traffic_oc.log; exit 1; }
  cp gpurun_out/${TAG}_traffic_oc/step_kernel_traffic.json $OUT/step_kernel_traffic.json
  bash tools/pmc_valu.sh ${TAG}_valu 262144 > $OUT/valu.log 2>&1 || { echo "valu failed"; tail -20 $OUT/valu.log; exit 1; }
  cp profiles/valu_issue.json $OUT/valu_issue.json
  echo "copy $OUT/step_kernel_traffic.json and $OUT/valu_issue.json into profiles/" ;;
C)
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  cut -c1-400 $OUT/bench.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o step -- python3 bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --collect-steps 0 --streaming-ring 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
  bash tools/all_configs.sh $OUT/all_configs.jsonl > $OUT/all_configs.txt 2>&1 || { echo "all_configs failed"; tail -20 $OUT/all_configs.txt; exit 1; }
  cat $OUT/all_configs.txt
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 tools/xchg_run_probe.py > $OUT/xchg.txt 2>&1 || { echo "xchg failed"; tail -20 $OUT/xchg.txt; exit 1; }
  tail -1 $OUT/xchg.txt ;;
esac
echo done
