#!/bin/bash
# Host-pointer (PCIe-inclusive) rates of the reference's call patterns: the Python ctypes patterns
# (scripts/pcie_rate.py) and the C++ facade's (tests/cpp/facade_rate.cpp), 200 frames each.
# usage (via gpurun): bash scripts/gpu_hostrate.sh <tag>
set -e
TAG=${1:-hostrate}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python3 scripts/pcie_rate.py --frames 200 > "$O/pcie_rate.json" 2> "$O/pcie_rate.err"
cat "$O/pcie_rate.json"
L=stereo_depth_ruler_amd/lib
g++ -std=c++17 -O2 -I include tests/cpp/facade_rate.cpp -L $L -lsdr -Wl,-rpath,$PWD/$L -o "$O/facade_rate"
timeout -k 10 60 python3 -c "
import sys; sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from test_gpu_facade_rate import write_inputs; write_inputs('$O')"
timeout -k 10 300 "$O/facade_rate" "$O" 200 > "$O/facade_rate.json"
cat "$O/facade_rate.json"
