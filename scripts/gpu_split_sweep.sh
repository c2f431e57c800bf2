set -o pipefail
for sp in 2048,1024 4096,2048 8192,4096 16384,4096; do
  echo "split $sp"; ORYX_ALS_SPLIT=$sp timeout -k 10 300 python scripts/als_kernel_bench.py --reps 3 || exit 1
done
