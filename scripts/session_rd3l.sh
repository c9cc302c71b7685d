#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
step diag_graphs 300 0 python -u scripts/diag_deq_graphs.py
bash "$(dirname "$0")/session_ab.sh"
