# Round 4, session 25: iovec AES-GCM in three length classes (16 / 8 / 4
# lanes), uniform short records at 4 lanes only on 64-byte runs: GPU suite,
# iov_bench at 1350 / 3000 / 4000 / 16384 B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s25
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -1 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step pytest_iov 300 python -u -m pytest tests/ -q -m gpu -k "iov" -rf --timeout 120 --timeout-method thread
for L in 1350 3000 4000 16384; do
  R=$(( 1414533120 / L ))
  step iov128_$L 200 python tools/iov_bench.py --aead aes-128-gcm --len $L --records $R --steps 20
  step iov256_$L 200 python tools/iov_bench.py --aead aes-256-gcm --len $L --records $R --steps 20
done
step pytest 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread
