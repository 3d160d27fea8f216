#!/bin/bash
# resident bf16 copies for the prefill GEMMs (default auto) vs scratch dequant per chunk
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_svd.py tests/test_video.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5_vid_gpu.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_pbf16_on.log 2>&1 || exit $?
LOCALAI_AMD_PREFILL_BF16=never timeout -k 10 500 python -u bench.py > gpurun_out/r5_pbf16_off.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_pbf16_on2.log 2>&1
