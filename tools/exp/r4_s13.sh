# Round 4, session 13: one-record GCM with the byte table of H^16 (16 lookups
# per GHASH step) and ChaCha iovec running pointers seeded at the record start
# and after a straddle: parity, latency against the previous build (ab_prev2),
# iovec rates against the previous ChaCha kernel (ab_chead).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s13
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
step par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_aead_api_gpu.py tests/test_bs16_total.py -q -m gpu -x -rf -k "(gcm and (kat or ref_edge or truncated or vector or extra or unaligned or tamper)) or iov or sealv or openv" --timeout 300 --timeout-method thread
for r in 1 2; do
  step latency_main_$r 200 python tools/latency_bench.py
  step latency_prev2_$r 200 env BSSL_AMD_LIB=$B/ab_prev2/libbssl_amd.so python tools/latency_bench.py
done
for r in 1 2; do
  step iov_chacha_main_$r 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
  step iov_chacha_chead_$r 200 env BSSL_AMD_LIB=$B/ab_chead/libbssl_amd.so python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
done
step iov_chacha_c00 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --cut1 0 --cut2 0
step iov_xchacha 200 python tools/iov_bench.py --aead xchacha20-poly1305 --records 1048576 --len 1350
step latency_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lat_prof -o lat -- python tools/latency_bench.py
