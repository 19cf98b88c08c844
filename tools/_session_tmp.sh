set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 900 bash tools/ab_envs.sh "DroneHoverBulletFreeEnvWithGust-v0:393216 DroneHoverBulletFreeEnvWithGust-v0:327680" build_ab/cur.so build_ab/nt_st.so 2>&1 | tee $O/ab_nt2.txt
