#!/bin/bash
# r05 closing check (third) on the committed build, the way the driver runs it: the
# whole -m gpu suite, smoke(), then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; print(g.smoke())" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -n 2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
exit $rc
