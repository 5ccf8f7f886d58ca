#!/bin/bash
# r03u: the JSON fast path's wave-count A/B, then the final build's GPU suite, smoke and bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_js_waves.sh || exit $?
bash tools/gpu_round.sh r03u quick || exit $?
tail -1 gpurun_out/bench_r03u.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; j=c["json_v2_ingest"]; print("C2", d["value"], d["ms_per_step"], c["step_roofline_frac"], "json", j["device_ms"], j["roofline_frac"], "C5", c["c5"]["ms_per_step"], c["c5"]["parity"])'
