#!/bin/bash
# A/B of the aux post-pass's parts on the C4-ext batches (tools/extprof.py): SG_DEBUG_FLAGS 1024 = no table
# updates, 2048 = no node commits (timing only: the node state is then wrong)
set -e
for f in 0 1024 2048 3072; do
  SG_DEBUG_FLAGS=$f timeout -k 10 300 python3 tools/extprof.py c4ext 3 2>&1 | grep c4ext | sed "s/^/flags=$f /"
done
