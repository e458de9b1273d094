set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/card_probe.py > gpurun_out/r5_card_probe.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_pytest_gpu.log 2>&1
echo "exit $?"
tail -3 gpurun_out/r5_pytest_gpu.log
