# Round 4, session 26: iovec AES-GCM three length classes (main) against two
# (ab_2way: < 4 KiB at 4 lanes), empty classes exit before the table build;
# 1M x 1350 B and 4000 B records, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s26
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -1 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
B=$PWD/boringssl_amd/csrc/build
step pytest_iov 300 python -u -m pytest tests/ -q -m gpu -k "iov or ragged or mixed" -rf --timeout 120 --timeout-method thread
for r in 1 2; do
  for v in main 2way; do
    if [ $v = main ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$B/ab_$v/libbssl_amd.so; fi
    step iov1350_${v}_$r 200 python tools/iov_bench.py --aead aes-128-gcm --len 1350 --records 1048576 --steps 20
    step iov3000_${v}_$r 200 python tools/iov_bench.py --aead aes-128-gcm --len 3000 --records 524288 --steps 20
  done
  unset BSSL_AMD_LIB
done
SPECS="config4:ab_2way" REPS="1 2" STEPS=10 step ab 400 bash tools/exp/ab_session.sh
cat $O/ab.log
