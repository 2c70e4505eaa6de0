#!/bin/bash
# The whole -m gpu suite (one pytest process), then smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-suite}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
exit $rc
