# Round-5 check of the final build on one GPU: smoke, the GPU suite, the
# single-record latency, key setup, the iovec rates.  Test failures do not
# stop the session; a crash, abort or time limit does.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5check}
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
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "[$(date +%T)] pytest rc=$rc" | tee -a $O/steps.log
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
step latency 200 python tools/latency_bench.py
step latency_c 120 tools/latency_c
step keysetup 200 python -u tools/keysetup_bench.py
step iov_gcm 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
step iov_gcm_1350 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
step iov_chacha 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
