#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash scripts/session_r05.sh gaps h43
head -45 gpurun_out/kt_h43_gaps.txt
