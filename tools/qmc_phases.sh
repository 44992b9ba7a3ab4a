#!/bin/bash
# GPU-box: qmc_kernel phase clocks with the -DBO_QMC_PHASES build (`make qmc-phases` -> ab_libs/libP.so)
# swapped in for the product library, which is restored afterwards.
set -u
cd "$GRAFT_REPO_ROOT"
cp botorch_amd/libbotorch_amd.so /tmp/libprod.so
cp ab_libs/libP.so botorch_amd/libbotorch_amd.so
timeout -k 10 240 python tools/qmc_phases.py
rc=$?
cp /tmp/libprod.so botorch_amd/libbotorch_amd.so
exit $rc
