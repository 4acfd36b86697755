#!/bin/bash
# instruction-class PMC of the LSTM and PWYX-RGB train passes after the row-mapped dW staging
cd $GRAFT_REPO_ROOT
bash tools/pmc_insts.sh r06dw_pmcinsts_lstm mspacman-lstm-figar > gpurun_out/c17_lstm.log 2>&1 && \
bash tools/pmc_insts.sh r06dw_pmcinsts_pwyx breakout-pwyx-figar-rgb > gpurun_out/c17_pwyx.log 2>&1
