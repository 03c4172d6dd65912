#!/bin/bash
# stage13 timing experiments (FR_STAGE_EXP 32/8/16/48) and wave-priority variants, same box
set -o pipefail
AB_CLASSES="stage layer3" bash tools/ab.sh "base e32 e8 e16 e48 p1 p2" 2 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
