#!/bin/bash
# The whole GPU suite and smoke(), as the driver runs them at round end.
set -o pipefail
out=gpurun_out/${1:-r03_suite}
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/pytest.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
