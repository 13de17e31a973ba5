#!/bin/sh
# Regenerates tests/golden/golden.{bin,json} from the reference's own
# CalculateChecksum (include/tcp-header.h:252-263).  Build container only:
# needs /root/reference.  The binary is written to /tmp, never committed.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REF=${REF:-/root/reference}
g++ -std=c++17 -O1 -Wall -I"$REF/include" -o /tmp/tcpck_gen_golden "$HERE/gen_golden.cc"
/tmp/tcpck_gen_golden "$HERE"
# Segmentation fixtures: the reference's data-segment send path
# (tcp-buffer.h:82-98, state.cc:167-184, socket-internal.h:186-199,
# socket-manager.h:259-260) on known send streams.
g++ -std=c++17 -O1 -Wall -I"$REF/include" -o /tmp/tcpck_gen_segment "$HERE/gen_segment.cc"
/tmp/tcpck_gen_segment "$HERE" 2>/dev/null
# Receive-path fixtures: wire images from the reference's send side, then
# ReceivePacket's verdict + TcpHeaderN2H (socket-manager.h:181-184).
g++ -std=c++17 -O1 -Wall -I"$REF/include" -o /tmp/tcpck_gen_receive "$HERE/gen_receive.cc"
/tmp/tcpck_gen_receive "$HERE"
