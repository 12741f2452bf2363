# Round 4, session 8: one-record kernel v2 (all record loads first, the tag's
# key-only part on wave 1, H^17 weights) + pinned host-memory flag variants
# for the single-record path; GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s8
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
step latency_main 300 python tools/latency_bench.py
for v in hmA hmC hmD hmE sq ev; do
  step latency_$v 300 env BSSL_AMD_LIB=$B/ab_$v/libbssl_amd.so python tools/latency_bench.py
done
step latency_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lat_prof -o lat -- python tools/latency_bench.py
step par_c_w4split 300 env BSSL_AMD_LIB=$B/ab_c_w4split/libbssl_amd.so python bench.py --config config3 --steps 2 --warmup 1 --no-cpu-baseline
step par_c_split 300 env BSSL_AMD_LIB=$B/ab_c_split/libbssl_amd.so python bench.py --config config3 --steps 2 --warmup 1 --no-cpu-baseline
SPECS="config3:ab_c_split,ab_c_w4split,ab_c_w4 config3x:ab_c_split,ab_c_w4split" REPS="1" STEPS=20 step ab 900 bash tools/exp/ab_session.sh
cat $O/ab.log
step iov_gcm 300 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
step iov_gcm_1350 300 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
step iov_chacha 300 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step lat_g1 300 env BSSL_AMD_LIB=$B/ab_g1/libbssl_amd.so python tools/latency_bench.py
step par_g1 600 env BSSL_AMD_LIB=$B/ab_g1/libbssl_amd.so python -u -m pytest tests/test_gpu_parity.py tests/test_aead_api_gpu.py -q -m gpu -x -rf -k "gcm and (kat or ref_edge or truncated or vector)" --timeout 300 --timeout-method thread
export BSSL_AMD_LIB=$B/ab_c1/libbssl_amd.so
step par_c1 600 python -u -m pytest tests/test_gpu_parity.py tests/test_aead_api_gpu.py tests/test_tls_golden.py -q -m gpu -x -rf -k "chacha or kat or ref_edge" --timeout 300 --timeout-method thread
step lat_c1 300 python tools/latency_bench.py
step lat_c1_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lat_prof_c1 -o lat -- python tools/latency_bench.py
