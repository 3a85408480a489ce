"""NGA packet constants and helpers -- mirror of src/common/header_config.py and
src/common/NGAPacket.py, following the switch's own layout (headers.p4:27-80).

Bulk pack/unpack runs on the device (ina_amd.ops.pack_nga / unpack_nga).  The
host helpers here parse or build single headers for control-path use (acks,
end markers, logging), the role NGAHeader plays at NGAPacket.py:62-102.

Layout note: the reference's ctypes NGAHeader assumes a 36-byte IP+NGA header
(HEADER_BYTE, header_config.py:5) and reads the payload as native-endian c_int
(NGAPacket.py:105-118); the wire (headers.p4) has a 15-byte NGA header after a
20-byte IPv4 header (35 bytes) and big-endian bit<32> payload words.  This
module follows the wire.
"""
from __future__ import annotations

import struct

from ._lib import (FLAG_ACK, FLAG_COLLISION, FLAG_OVERFLOW, FLAG_RESEND,  # noqa: F401
                   NGA_HDR_BYTES, NUM_REGISTER)

# header_config.py:1-19
NGA_TYPE = 0x0012
IPV4_HEADER_BYTE = 20
HEADER_BYTE = IPV4_HEADER_BYTE + NGA_HDR_BYTES   # 35 on the wire (the reference says 36)
WORKERMAPBIT, DEGREEBIT = 32, 8
OVERFLOWBIT = ISACKBIT = ECNBIT = RESENDBIT = 1
TIMEBIT, INDEXBIT, SWITCHIDBIT, SEQUENCEBIT = 4, 32, 8, 32
DATA_NUM = 32            # values per packet in the P4 program (ngaa_payload_h)
DATA_BYTE = 4 * DATA_NUM

_HDR = struct.Struct("!IBBIBI")   # DataManager.py:122-130 packs '!IbbIbI' (same bytes)


def build_header(bitmap: int, count: int, flags: int, index: int, switch_id: int,
                 frag_id: int) -> bytes:
    """15-byte ngaa_h (headers.p4:27-38)."""
    return _HDR.pack(bitmap & 0xFFFFFFFF, count & 0xFF, flags & 0xFF, index & 0xFFFFFFFF,
                     switch_id & 0xFF, frag_id & 0xFFFFFFFF)


def end_marker(worker_id: int, degree: int, switch_id: int) -> bytes:
    """Header-only end-of-stream datagram (DataManager.py:155-164): index 0, seq 0."""
    return build_header(worker_id, degree, 0, 0, switch_id, 0)


def ack_for(header: bytes) -> bytes:
    """PS ack for a completed slot: same index / frag, is_ack=1 (fragcheck.p4:26-31)."""
    f = parse_header(header)
    return build_header(f["bitmap"], f["count"], FLAG_ACK, f["index"], f["switch_id"],
                        f["frag_id"])


def parse_header(buf: bytes, offset: int = 0) -> dict:
    """Fields of one ngaa_h starting at `offset` (use offset=20 on a raw IPv4 datagram)."""
    bitmap, count, flags, index, sw, frag = _HDR.unpack_from(buf, offset)
    return {"bitmap": bitmap, "count": count, "flags": flags,
            "overflow": flags >> 7 & 1, "is_ack": flags >> 6 & 1, "collision": flags >> 5 & 1,
            "resend": flags >> 4 & 1, "timestamp": flags & 0xF,
            "index": index, "switch_id": sw, "frag_id": frag}


def packet_bytes(V: int = DATA_NUM) -> int:
    return NGA_HDR_BYTES + 4 * V
