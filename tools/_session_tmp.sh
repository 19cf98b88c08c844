set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in full_pw1 full_pw3; do
  CF2SIM_LIB=build_ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_rollout_fused.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; echo "$v rc=$?"; tail -3 $O/pytest_$v.log
done
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "intree rc=$?"; tail -3 $O/pytest_gpu.log
timeout -k 10 900 bash tools/ab_envs.sh "DroneHoverBulletFreeEnvWithConstWind-v0:4096 DroneHoverBulletFreeEnvWithGust-v0:32768" build_ab/hd_prev.so build_ab/nofin.so build_ab/bal.so 2>&1 | tee $O/ab.txt
timeout -k 10 900 bash tools/ab_envs.sh "DroneHoverBulletFreeEnvWithGust-v0:262144 DroneHoverBulletFreeEnvWithGust-v0:1048576" build_ab/bal.so build_ab/nt_ld.so build_ab/nt_st.so build_ab/nt_both.so 2>&1 | tee $O/ab_nt.txt
