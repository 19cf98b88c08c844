set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab1
timeout -k 10 200 python tools/donerate.py > gpurun_out/ab1/done.txt 2>&1 || exit 1
cat gpurun_out/ab1/done.txt
SKIP_TESTS=1 bash tools/ab_run.sh build_ab/base.so build_ab/noreset.so build_ab/noresetmath.so || exit 1
CF2SIM_LIB=build_ab/timing.so timeout -k 10 200 python tools/timeline.py --envs 262144 > gpurun_out/ab1/tl262k.txt 2>&1 || exit 1
CF2SIM_LIB=build_ab/timing.so timeout -k 10 200 python tools/timeline.py --envs 16384 > gpurun_out/ab1/tl16k.txt 2>&1 || exit 1
cat gpurun_out/ab1/tl262k.txt gpurun_out/ab1/tl16k.txt
