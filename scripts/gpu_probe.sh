#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
CFG=5 timeout -k 5 120 python tools/gemm_layout_probe.py 2>&1 | grep -v amdgpu.ids
CFG=6 timeout -k 5 120 python tools/gemm_layout_probe.py 2>&1 | grep -v amdgpu.ids
