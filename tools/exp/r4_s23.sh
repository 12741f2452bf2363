# Round 4, session 23: the iovec length split on the whole GPU suite, and
# iov_bench at the round-4 table's sizes (1M x 1350 B, 256K x 16 KiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s23
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
for r in 1 2; do
  step iov_128_1350_$r 200 python tools/iov_bench.py --aead aes-128-gcm --len 1350 --records 1048576 --steps 20
  step iov_256_1350_$r 200 python tools/iov_bench.py --aead aes-256-gcm --len 1350 --records 1048576 --steps 20
done
step iov_128_4000 200 python tools/iov_bench.py --aead aes-128-gcm --len 4000 --records 524288 --steps 20
step iov_128_16384 200 python tools/iov_bench.py --aead aes-128-gcm --len 16384 --records 262144 --steps 20
step pytest 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread
