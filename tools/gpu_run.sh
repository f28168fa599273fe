set -o pipefail
timeout -k 10 400 python -m pytest -q tests/test_gpu_trainer.py tests/test_gpu_configs.py -k "stepper or position_csr or fixed_cotangent" 2>&1 | tail -5
