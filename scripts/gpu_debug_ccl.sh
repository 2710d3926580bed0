#!/bin/bash
cd "$(dirname "$0")/.."
export SSA_NO_AUTOBUILD=1 PYTHONPATH=$PWD
timeout -k 10 120 python scripts/debug_ccl.py 2>&1 | grep -v amdgpu.ids | head -60
