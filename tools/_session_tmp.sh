set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 bash tools/ab_envs.sh "DroneHoverBulletFreeEnvWithConstWind-v0:4096 DroneHoverBulletFreeEnvWithGust-v0:32768" build_ab/merge2.so build_ab/post1.so build_ab/p1pre.so build_ab/post3.so 2>&1 | tee $O/ab.txt
