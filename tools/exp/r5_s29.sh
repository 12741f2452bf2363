# Round-5 session 29: ChaCha20-Poly1305 iovec records with the store anchor
# handed over by the load cursor (the build) against without (ab_cho0).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s29}
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
step pytest_chacha_iov 400 python -u -m pytest tests/ -q -m gpu -k "iov or chacha or aead_api or ref_edge" -x --timeout 120 --timeout-method thread
for rep in 1 2; do
for v in base cho0; do
  if [ $v = base ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$C/ab_$v/libbssl_amd.so; fi
  step ${v}_1350_$rep 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350
  step ${v}_16k_$rep 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 131072 --len 16384
  step ${v}_x1350_$rep 200 python tools/iov_bench.py --aead xchacha20-poly1305 --records 1048576 --len 1350
done
done
