# Round 4, session 11: completion-word polling for single records, 16 lanes
# per record for iovec / unaligned GCM batches, one-chunk AD fast path:
# GPU suite, latency against the previous build, iovec rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s11
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
# (test failures do not stop the session; a crash, abort or time limit does)
echo "[$(date +%T)] pytest" | tee -a $O/steps.log
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "[$(date +%T)] pytest rc=$rc" | tee -a $O/steps.log
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
step latency_main 200 python tools/latency_bench.py
step latency_prev 200 env BSSL_AMD_LIB=$B/ab_prev/libbssl_amd.so python tools/latency_bench.py
step latency_main2 200 python tools/latency_bench.py
step latency_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lat_prof -o lat -- python tools/latency_bench.py
step iov_gcm 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
step iov_gcm_1350 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
step iov_chacha 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_xchacha 200 python tools/iov_bench.py --aead xchacha20-poly1305 --records 1048576 --len 1350
step iov_chacha_16k 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 131072 --len 16384
step iov_siv 200 python tools/iov_bench.py --aead aes-128-gcm-siv --records 262144 --len 16384
for c in config2 configG config4; do step bench_$c 200 python bench.py --config $c --no-cpu-baseline; done
