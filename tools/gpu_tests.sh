timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r2b.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu_r2b.txt
