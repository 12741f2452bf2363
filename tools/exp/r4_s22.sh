# Round 4, session 22: iovec AES-GCM batches in length order split into a
# long-record launch (16 lanes) and a short-record launch (4 lanes): iovec
# parity tests, iov_bench at 1350 B and 16 KiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s22
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -2 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_iov 300 python -u -m pytest tests/ -q -m gpu -k "iov" -rf --timeout 120 --timeout-method thread
for L in 1350 16384; do
  R=$(( L == 1350 ? 2097152 : 262144 ))
  for a in aes-128-gcm aes-256-gcm; do
    step iov_${a}_$L 200 python tools/iov_bench.py --aead $a --len $L --records $R --steps 10
  done
done
