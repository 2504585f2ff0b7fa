#!/bin/bash
# Round-4 flakiness check: the whole GPU suite twice in a row on one box.
set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:randomly > $O/gpu_tests_flaky1.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:randomly > $O/gpu_tests_flaky2.txt 2>&1 || exit 2
echo all done
