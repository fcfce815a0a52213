#!/bin/bash
set -u
BATCHES='22 23 24 25' bash scripts/sweep_batch.sh || exit 1
WORKLOAD=config3 BATCHES='8 12 16 20 24' bash scripts/sweep_batch.sh || exit 1
WORKLOAD=config5 BATCHES='12 16 24 32' bash scripts/sweep_batch.sh || exit 1
