# Round-5 session 26: AES-GCM iovec records with the lane's first block loaded
# before the record setup (ab_ie1, -DGCM_IOV_EARLY=1) against the build.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s26}
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
BSSL_AMD_LIB=$C/ab_ie1/libbssl_amd.so step ie1_pytest_iov 300 python -u -m pytest tests/ -q -m gpu -k "iov" -x --timeout 120 --timeout-method thread
for rep in 1 2; do
for v in base ie1; do
  if [ $v = base ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$C/ab_$v/libbssl_amd.so; fi
  step ${v}_16k_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
  step ${v}_1350_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350
  step ${v}_3000_$rep 200 python tools/iov_bench.py --aead aes-128-gcm --records 524288 --len 3000
done
done
