# Round-5 session 24: where the iovec batches lose against contiguous records
# (kernel trace of tools/iov_bench.py; aligned-chunk variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s24}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -1 "$O/$name.log" | tee -a $O/steps.log
  [ $rc -eq 0 ] || exit $rc
}
step gcm16k 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384
step gcm16k_al 200 python tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384 --cut1 16 --in-gap 0 --out-gap 0
step gcm1350_al 200 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350 --cut1 16 --cut2 672 --in-gap 10 --out-gap 10
step chacha_al 200 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --cut1 64 --cut2 640 --in-gap 10 --out-gap 10
step prof_gcm16k 300 rocprofv3 --kernel-trace --stats -d $O/prof_gcm16k -o run -- python3 tools/iov_bench.py --aead aes-128-gcm --records 262144 --len 16384 --steps 5
step prof_gcm1350 300 rocprofv3 --kernel-trace --stats -d $O/prof_gcm1350 -o run -- python3 tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350 --steps 5
step prof_chacha 300 rocprofv3 --kernel-trace --stats -d $O/prof_chacha -o run -- python3 tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --steps 5
