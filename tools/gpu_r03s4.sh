#!/bin/bash
# stage13 trivial-epilogue timing (e8), priority alternation (p2), layer2 split-stage epilogue/exchange timing
set -o pipefail
AB_CLASSES="stage layer3,stage layer2,stage layer1" bash tools/ab.sh "base e8 e8p2 p2 e32 s4 s2" 2 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
