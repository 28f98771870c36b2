#!/bin/bash
# Round 3 measurements: config 5 (native S3 front) and the durable write path A/B.
set -o pipefail
bash scripts/gpu_s3.sh && bash scripts/gpu_durable.sh
