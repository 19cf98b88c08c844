set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r03b/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r03b/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03b/pytest_gpu.log
timeout -k 10 600 bash tools/ab_envs.sh "DroneHoverBulletFreeEnvWithConstWind-v0:4096 DroneHoverBulletFreeEnvWithGust-v0:16384 DroneHoverBulletFreeEnvWithGust-v0:32768 DroneHoverBulletFreeEnvWithGust-v0:262144" build_ab/small_old.so build_ab/small_new.so 2>&1 | tee gpurun_out/r03b/ab_small.txt
