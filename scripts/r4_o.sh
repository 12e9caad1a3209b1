#!/bin/bash
# round 4 (o): reconcile with coalesced first-64-B stores (four lanes per frame) vs field stores
source scripts/lib_steps.sh
step recon_tests 400 python -u -m pytest tests/test_reconcile_gpu.py -x -q --timeout 120 --timeout-method thread
export AB_STEPS=1000
step recon_ab 170 bash scripts/ab_variants.sh "reconcile64 reconcile_imix" "FETCH_SIZE;WRITE_SIZE" recon_fields recon_coal
