#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/con; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
L=disturbance-crazyfile-simulation_amd/cf2sim/libcf2sim.so
bash tools/ab_envs.sh "DroneHoverBulletFreeEnvWithGust-v0:262144 DroneHoverBulletFreeEnvWithGust-v0:32768 DroneHoverBulletFreeEnvWithConstWind-v0:4096 DroneHoverBulletFreeEnvWithGust-v0:1048576" $L build_ab/fast_contract.so > $O/ab.txt 2>&1
cat $O/ab.txt
