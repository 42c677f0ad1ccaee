O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" > $O/status
