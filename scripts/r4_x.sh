#!/bin/bash
# round 4 (x): where reconcile64's time goes: without frame stores, without the status store
source scripts/lib_steps.sh
export AB_STEPS=1000
step ab 300 bash scripts/ab_variants.sh "reconcile64" "-" rc_base rc_nostore rc_nostatus rc_base
