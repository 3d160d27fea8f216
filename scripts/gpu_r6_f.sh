export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tp_sample_gpu.py > gpurun_out/r6f_tps.log 2>&1; tail -15 gpurun_out/r6f_tps.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tp_gpu.py -s -k "True-False-True" > gpurun_out/r6f_tpe.log 2>&1; grep -E "TP_ROWS|passed|failed|Error|error" gpurun_out/r6f_tpe.log | tail -15
