# Round 4, session 24: lanes for short records off 64-byte runs.  main: 4
# lanes for uniform records <= 4 KiB only when records start on 64-byte
# boundaries (else 8), short iovec records at 4 lanes; ab_l4any: 4 lanes at
# any alignment (the previous rule); ab_iov8: short iovec records at 8 lanes.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s24
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
for r in 1 2; do
  for v in main l4any iov8; do
    if [ $v = main ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$B/ab_$v/libbssl_amd.so; fi
    step iov1350_${v}_$r 200 python tools/iov_bench.py --aead aes-128-gcm --len 1350 --records 1048576 --steps 20
    step iov4000_${v}_$r 200 python tools/iov_bench.py --aead aes-128-gcm --len 4000 --records 524288 --steps 20
  done
  unset BSSL_AMD_LIB
done
SPECS="configG:ab_l4any" REPS="1 2" STEPS=20 step ab 400 bash tools/exp/ab_session.sh
cat $O/ab.log
