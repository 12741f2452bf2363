set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for c in "5 -1" "64 -1" "64 640" "0 0" "5 5"; do
    set -- $c
    echo "== $rep cut1=$1 cut2=$2"; timeout -k 10 120 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 --cut1 $1 --cut2 $2 || exit 1
  done
  echo "== $rep gcm"; timeout -k 10 120 python tools/iov_bench.py --aead aes-128-gcm --records 1048576 --len 1350 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/s20.txt
