set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab4
for lib in tl_one tl_roles; do for n in 4096 262144; do
  echo "=== $lib N=$n"; CF2SIM_LIB=build_ab/$lib.so timeout -k 10 200 python tools/timeline.py --envs $n 2>&1 | grep -v amdgpu.ids || exit 1
done; done
