#!/bin/bash
tools/gpu_steps.sh conv_tests 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "conv or linear" -p no:cacheprovider --- bench_conv 400 python tools/bench_conv.py
