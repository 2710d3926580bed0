#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 PYTHONPATH=$PWD
r() { SSA_POST_STAGES=$1 timeout -k 10 120 python scripts/debug_post_graph.py graph 2 flat > gpurun_out/dbg_post_$1.log 2>&1; local rc=$?; echo "== stages=$1 rc=$rc"; grep -E "replay|eager|Error" gpurun_out/dbg_post_$1.log | head -5; return $rc; }
r 99
