#!/bin/bash
# several measurement scripts in one GPU call (each under its own time limit inside)
bash scripts/attn_fused_ab.sh && bash scripts/gemm_ksweep.sh
