#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_r2_speed2.sh
