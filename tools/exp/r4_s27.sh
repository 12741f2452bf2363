# Round 4, session 27: the final build with the iovec length classes and the
# 64-byte-run rule for 4 lanes: GPU suite, smoke, default bench, configs G/4,
# iov_bench at 1350 / 3000 / 16384 B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s27
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -1 "$O/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step bench_configG 200 python bench.py --config configG --no-cpu-baseline
step bench_config4 200 python bench.py --config config4 --no-cpu-baseline
step iov1350 200 python tools/iov_bench.py --aead aes-128-gcm --len 1350 --records 1048576 --steps 20
step iov3000 200 python tools/iov_bench.py --aead aes-128-gcm --len 3000 --records 524288 --steps 20
step iov16384 200 python tools/iov_bench.py --aead aes-128-gcm --len 16384 --records 262144 --steps 20
step pytest 600 python -u -m pytest tests/ -q -m gpu -rf --timeout 300 --timeout-method thread
