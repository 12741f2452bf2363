# Round 4, session 14: one-record GCM in two shapes (256 threads + nibble
# table up to 4 KiB, 1024 threads + byte table above), GCM iovec pointers
# seeded at the unit start: parity, latency and iovec rates against the
# previous build (ab_prev2).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s14
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
step par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_aead_api_gpu.py tests/test_bs16_total.py tests/test_tls_golden.py -q -m gpu -x -rf -k "gcm or iov or sealv or openv" --timeout 300 --timeout-method thread
for r in 1 2 3; do
  step latency_main_$r 200 python tools/latency_bench.py
  step latency_prev2_$r 200 env BSSL_AMD_LIB=$B/ab_prev2/libbssl_amd.so python tools/latency_bench.py
done
for r in 1 2; do
  step iov_gcm_main_$r 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
  step iov_gcm_prev2_$r 200 env BSSL_AMD_LIB=$B/ab_prev2/libbssl_amd.so python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
done
step iov_gcm_a05 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384 --in-gap 0 --out-gap 0
step latency_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lat_prof -o lat -- python tools/latency_bench.py
