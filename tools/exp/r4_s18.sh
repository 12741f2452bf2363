# Round 4, session 18: record memory through global pointers (no flat
# accesses in the iovec walks and the partial-block / tag paths): GPU suite,
# bench lines of configs 2, G, 3, 4, 5, iovec rates, latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s18
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
echo "[$(date +%T)] pytest" | tee -a $O/steps.log
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "[$(date +%T)] pytest rc=$rc" | tee -a $O/steps.log
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for c in config2 configG config3 config4 config5; do step bench_$c 200 python bench.py --config $c --no-cpu-baseline; done
step iov_gcm 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
step iov_gcm_prev2 200 env BSSL_AMD_LIB=$B/ab_prev2/libbssl_amd.so python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
step iov_gcm_1350 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
step iov_chacha 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_chacha_prev2 200 env BSSL_AMD_LIB=$B/ab_prev2/libbssl_amd.so python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
step iov_xchacha 200 python tools/iov_bench.py --aead xchacha20-poly1305 --records 1048576 --len 1350
step iov_chacha_16k 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 131072 --len 16384
step iov_siv 200 python tools/iov_bench.py --aead aes-128-gcm-siv --records 262144 --len 16384
step latency_c 120 tools/latency_c
SPECS="config2:ab_prev2 configG:ab_prev2 config4:ab_prev2" REPS="1" STEPS=10 step ab 400 bash tools/exp/ab_session.sh
cat $O/ab.log
