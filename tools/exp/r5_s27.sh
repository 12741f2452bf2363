# Round-5 session 27: SQ counters of the AES-GCM and ChaCha20-Poly1305 iovec
# kernels beside the contiguous kernels on the same records (iov_bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s27}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  [ $rc -eq 0 ] || { tail -n 3 "$O/$name.log"; exit $rc; }
}
SQ="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VMEM"
step sq_gcm16k 200 rocprofv3 --kernel-include-regex "gcm_kernel" --pmc $SQ -d $O/sq_gcm16k -o run --output-format csv -- python3 tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384 --steps 2
step sq_gcm1350 200 rocprofv3 --kernel-include-regex "gcm_kernel" --pmc $SQ -d $O/sq_gcm1350 -o run --output-format csv -- python3 tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350 --steps 2
step sq_chacha 200 rocprofv3 --kernel-include-regex "chacha_poly_kernel" --pmc $SQ -d $O/sq_chacha -o run --output-format csv -- python3 tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --steps 2
