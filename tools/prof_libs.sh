# rocprofv3 kernel stats of the bench for each library build given.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_libs
for lib in "$@"; do
  name=$(basename $lib .so)
  CF2SIM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_libs/$name -o p -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_libs/$name.json 2> gpurun_out/prof_libs/$name.err || { echo "rocprof failed $lib"; tail -5 gpurun_out/prof_libs/$name.err; exit 1; }
  echo "== $name"
  f=$(find gpurun_out/prof_libs/$name -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'cf2' in r['Name']: print('%-40s calls %5s avg %8.1f us min %8.1f max %8.1f' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
"
done
