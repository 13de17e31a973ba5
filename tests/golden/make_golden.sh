#!/bin/sh
# Regenerates tests/golden/golden.{bin,json} from the reference's own
# CalculateChecksum (include/tcp-header.h:252-263).  Build container only:
# needs /root/reference.  The binary is written to /tmp, never committed.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REF=${REF:-/root/reference}
g++ -std=c++17 -O1 -Wall -I"$REF/include" -o /tmp/tcpck_gen_golden "$HERE/gen_golden.cc"
/tmp/tcpck_gen_golden "$HERE"
