# Round-5 session 30: AES-GCM iovec records with the load cursor keeping its chunk end
# (ab_ke1, GCM_IOV_KEEP_END=1) against without (the build).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s30}
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
BSSL_AMD_LIB=$C/ab_ke1/libbssl_amd.so step pytest_iov_gcm 400 python -u -m pytest tests/ -q -m gpu -k "iov or gcm or aead_api or ref_edge" -x --timeout 120 --timeout-method thread
for rep in 1 2; do
for v in base ke1; do
  if [ $v = base ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$C/ab_$v/libbssl_amd.so; fi
  step ${v}_16k_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
  step ${v}_1350_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
  step ${v}_3000_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 524288 --len 3000
done
done
