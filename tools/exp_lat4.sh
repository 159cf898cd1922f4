#!/bin/bash
set -o pipefail
bash tools/exp_lat3.sh || exit 1
bash tools/exp_pmc1.sh l4c2 wgrad lattice_wgrad
