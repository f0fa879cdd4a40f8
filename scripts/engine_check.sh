mkdir -p gpurun_out/eng
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_chunked_prefill.py tests/test_hf_parity_gpu.py -m gpu > gpurun_out/eng/pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/eng/pytest.log; exit $rc
