# Round 4, session 9: ChaCha iovec last-block fast path (ci1): parity of the
# iovec and single-record cases, iovec and contiguous rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s9
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
B=$PWD/boringssl_amd/csrc/build
export BSSL_AMD_LIB=$B/ab_ci1/libbssl_amd.so
step par_ci1 600 python -u -m pytest tests/test_gpu_parity.py tests/test_aead_api_gpu.py -q -m gpu -x -rf -k "iov or sealv or openv" --timeout 300 --timeout-method thread
step iov_chacha_ci1 300 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_xchacha_ci1 300 python tools/iov_bench.py --aead xchacha20-poly1305 --records 1048576 --len 1350
unset BSSL_AMD_LIB
step iov_chacha_main 300 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
