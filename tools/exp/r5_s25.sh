# Round-5 session 25: lanes per record of the AES-GCM iovec length classes
# (ab_base: 16 / 8 / 4; ab_il8: 8 for >= 4 KiB; ab_is8: 8 below 2 KiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s25}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -n 1 "$O/$name.log" | tee -a $O/steps.log
  [ $rc -eq 0 ] || exit $rc
}
C=boringssl_amd/csrc/build
for rep in 1 2; do
for v in base il8 is8; do
  export BSSL_AMD_LIB=$C/ab_$v/libbssl_amd.so
  step ${v}_16k_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
  step ${v}_1350_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
  step ${v}_3000_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 524288 --len 3000
done
done
unset BSSL_AMD_LIB
for v in il8 is8; do
  BSSL_AMD_LIB=$C/ab_$v/libbssl_amd.so step ${v}_pytest_iov 300 python -u -m pytest tests/ -q -m gpu -k "iov" -x --timeout 120 --timeout-method thread
done
