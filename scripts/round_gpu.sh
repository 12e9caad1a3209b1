#!/bin/bash
# tests + bench + profiles in one gpurun call
bash scripts/gpu_check.sh || exit $?
bash scripts/profile.sh "$@"
