#!/bin/bash
# Round-3 end-of-round check of the committed tree (the two-wave dK/dV experiment this slot was
# reserved for was dropped before it ran): full GPU suite, smoke, bench, kernel stats.
bash "$(dirname "$0")/gpu_final_check.sh"
