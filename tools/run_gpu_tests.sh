set -o pipefail
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=25 -p no:cacheprovider > gpurun_out/hot2_pytest.log 2>&1 || exit 1
