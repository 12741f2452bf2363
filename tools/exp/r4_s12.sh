# Round 4, session 12: GPU suite + smoke on the final build; iovec chunk-cut
# breakdown for ChaCha (one chunk, block-aligned cuts, the default cuts).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s12
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
echo "[$(date +%T)] pytest" | tee -a $O/steps.log
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "[$(date +%T)] pytest rc=$rc" | tee -a $O/steps.log
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
step iov_chacha_c00 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --cut1 0 --cut2 0
step iov_chacha_c64 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --cut1 64 --cut2 640
step iov_chacha_c5 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_chacha_a00 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --cut1 0 --cut2 0 --in-gap 0 --out-gap 0
step iov_gcm_a05 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384 --in-gap 0 --out-gap 0
