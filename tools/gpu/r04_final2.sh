#!/bin/bash
# Round-4 final validation, second pass (after the nullable-key changes): same steps as r04_final.sh
export R04_FINAL_DIR=r04final2
bash tools/gpu/r04_final.sh
