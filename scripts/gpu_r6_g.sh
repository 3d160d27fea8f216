export PYTHONUNBUFFERED=1
python -c "from localai_amd.models import synth; synth.write_model('/tmp/tp.gguf', 'tiny-llama', exact=True)"
TP_REHEARSAL_SAMPLING=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 scripts/tp_rehearsal.py /tmp/tp.gguf > gpurun_out/r6g.log 2>&1; echo rc=$?
grep -v "^\[Gloo\]" gpurun_out/r6g.log | grep -B2 -A25 "Traceback" | head -80
grep "TP_ROWS\|TP_OK\|TP texts" gpurun_out/r6g.log
