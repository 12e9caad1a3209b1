#!/bin/bash
# round 4 (v): reconcile with the four rounds' re-reads issued together, against the previous build
source scripts/lib_steps.sh
step recon_tests 400 python -u -m pytest tests/test_reconcile_gpu.py -x -q --timeout 120 --timeout-method thread
export AB_STEPS=1000
step ab 300 bash scripts/ab_variants.sh "reconcile64 reconcile_imix" "-" cur recon4 cur recon4
