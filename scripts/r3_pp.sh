#!/bin/bash
# stream path with the next load group issued before the current one is summed
source scripts/lib_steps.sh
step parse_tests 600 python -u -m pytest tests/test_parse_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread
step ab 900 bash scripts/ab_variants.sh "imix_csum parse256" "SQ_INSTS_VALU SQ_WAVES" base pp1
step ab2 600 bash scripts/ab_variants.sh "imix_csum" "-" pp1 base pp1 base
