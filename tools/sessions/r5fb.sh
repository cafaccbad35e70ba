#!/bin/bash
# r5 final check, part b: cfg 5 'N' / 'T' and cfg 3 / cfg 4 kernel traces and HBM traffic passes
# (tools/c5_pmc.sh, tools/c34_prof.sh) -> profiles/r5f2
set -o pipefail
tools/c5_pmc.sh r5f2_c5pmc || exit 1
tools/c34_prof.sh r5f2_c34 || exit 1
