# Round 4, session 10: the working-tree build as main (one-record ChaCha and
# GCM kernels v3, ChaCha iovec last-block and two-chunk straddle paths): GPU suite, single-record
# latency against the previous build (ab_prev) and its host-memory / sync
# variants, iovec rates, the ChaCha occupancy A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s10
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
for v in prev sq ev hmA hmC hmD hmE; do
  step latency_$v 200 env BSSL_AMD_LIB=$B/ab_$v/libbssl_amd.so python tools/latency_bench.py
done
step iov_gcm 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
step iov_gcm_1350 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
step iov_chacha 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_chacha_prev 200 env BSSL_AMD_LIB=$B/ab_prev/libbssl_amd.so python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_chacha_ci1 200 env BSSL_AMD_LIB=$B/ab_ci1/libbssl_amd.so python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_chacha_2 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step latency_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lat_prof -o lat -- python tools/latency_bench.py
SPECS="config3:ab_c_split,ab_c_w4split,ab_c_w4" REPS="1" STEPS=20 step ab 400 bash tools/exp/ab_session.sh
cat $O/ab.log
