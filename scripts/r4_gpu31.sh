set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/serving_path_profile.py > gpurun_out/r4_serving_path_profile_v2.txt 2> gpurun_out/r4_serving_path_profile_v2.err || exit 1
echo done
