#!/bin/bash
# Build tools/solvebench on the box (the binary is not pushed) and run it:
# the one-wave solve variants' latency, bitwise checks, fp64 latency probes.
set -o pipefail
make -C tools solvebench > /dev/null && timeout -k 10 300 tools/solvebench
