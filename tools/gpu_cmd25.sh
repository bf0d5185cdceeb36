#!/bin/bash
set -u
for i in 1; do timeout -k 10 300 python -u -m pytest tests/test_half.py -m gpu -q --timeout 200 --timeout-method thread -k "minibatch_gradient" -s 2>&1 | grep -E "torch-fp32|passed|failed" ; done
