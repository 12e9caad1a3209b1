#!/bin/bash
# stream path with wave-uniform start masks + 64-bit chunk masks: parity, A/B
source scripts/lib_steps.sh
step parse_tests 600 python -u -m pytest tests/test_parse_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread
step ab 900 bash scripts/ab_variants.sh "imix_csum parse256 parse1500" "SQ_INSTS_VALU SQ_WAVES" base sm3 sm3m
step ab2 600 bash scripts/ab_variants.sh "imix_csum parse256" "-" sm3m base sm3m base
