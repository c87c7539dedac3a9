#!/bin/bash
set -o pipefail
bash tools/gpu_r03r.sh && bash tools/gpu_r03s.sh
