set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcpol; mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*\|TCP_[A-Z_0-9]*\|GRBM_[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/names.txt
grep -i "mfma\|lds\|valu\|busy\|wait" $OUT/names.txt | head -80
