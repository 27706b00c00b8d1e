cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "golden" > gpurun_out/pytest_gpu.log 2>&1; echo "rc=$?"
