#!/bin/bash
# RangeDeps half of acc_partial_deps_batch on a child context thread (concurrent with the KeyDeps half); mixed-path
# offset scans in one launch; g + prep slots one fill; bumped-committed maxima one scan; big list from the mark pass:
# full GPU suite, config 4 A/B (fused, mixed) against r4base and the serial switch, config 2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests > gpurun_out/r4r_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4r_tests.log; [ $rc -eq 0 ] || exit $rc
CFGS=4 STEPS=3 bash tools/gpu_abn.sh new new+ACC_PD_SERIAL=1 r4base || exit 1
CFGS=2 STEPS=20 bash tools/gpu_abn.sh new r4base || exit 1
