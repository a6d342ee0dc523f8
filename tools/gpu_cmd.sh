#!/bin/bash
# scratch GPU session script (the command of the last gpurun call): L/14 leg with the large-STORE
# GEMMs on G4 (config 13) vs config 1, alternating
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
VARIANTS="c1a:CLM_G4_STORE=0;g4a:CLM_G4_STORE=1;c1b:CLM_G4_STORE=0;g4b:CLM_G4_STORE=1" bash tools/l14_ab.sh
