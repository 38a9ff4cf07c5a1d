#!/bin/bash
for d in 64 192 320 448; do
  echo "dbg=$d: "; SGD_DBG=$d timeout -k 10 120 python3 tools/prof_c2.py 3 2>&1 | grep -E "advance ms|stamps" || exit 1
done
