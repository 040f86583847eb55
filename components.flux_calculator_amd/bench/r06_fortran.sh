#!/bin/bash
# round 6: the Fortran drop-in host in every mode (fcx_commit_engine now audits every plan
# with fcx_plan_check first) and the selftest of the full iso_c_binding interface set.
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/fortran}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_fortran.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/test.log 2>&1; rc=$?
echo "fortran rc=$rc" | tee $O/steps.txt
exit $rc
