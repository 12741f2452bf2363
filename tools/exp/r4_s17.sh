# Round 4, session 17: PMC of the ChaCha iovec kernel against the unaligned
# contiguous (ANY) kernel on the same records (tools/iov_bench.py, one chunk
# per record and the default three chunks).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s17
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
for cut in "0 0" "5 675"; do
  set -- $cut
  tag=c$1
  B="python3 tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --steps 3 --cut1 $1 --cut2 $2"
  step pmc_sq_$tag 200 rocprofv3 --kernel-include-regex chacha_poly_kernel --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $O/pmc_sq_$tag -o run --output-format csv -- $B
  step pmc_sq2_$tag 200 rocprofv3 --kernel-include-regex chacha_poly_kernel --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH -d $O/pmc_sq2_$tag -o run --output-format csv -- $B
  step pmc_fetch_$tag 200 rocprofv3 --kernel-include-regex chacha_poly_kernel --pmc FETCH_SIZE -d $O/pmc_fetch_$tag -o run --output-format csv -- $B
  step stats_$tag 200 rocprofv3 --kernel-trace --stats -d $O/stats_$tag -o run --output-format csv -- $B
done
