"""Control-plane wire format.

Reference (packets.py:9-92): a fixed 33 040-byte struct ("i255s6si32768s") per
datagram — every message is IP-fragmented, and a JSON payload over 32 KiB is
silently truncated so ``unpack`` fails and the packet is dropped (a
WORKER_TASK_REQUEST overflows at ~122 images).

Here: a small binary header + JSON payload, and messages larger than one MTU
are split into MTU-sized fragments that the receiver reassembles, so nothing
relies on IP fragmentation and there is no payload cap. Every frame carries a
request id (``seq``) so replies resolve per-request futures instead of the
reference's single shared wait slot (worker.py:43-44, 1123-1135).

Header (big-endian): magic 'DM' | ver u8 | type u16 | flags u8 | seq u64 |
frag_idx u16 | frag_cnt u16 | msg_id u32 | sender_len u8 | sender | payload.
"""
from __future__ import annotations

import json
import struct
import time
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Any, Dict, List, Optional, Tuple

MAGIC = b"DM"
VERSION = 1
_HDR = struct.Struct(">2sBHBQHHIB")
MTU_PAYLOAD = 1200  # bytes of body per datagram fragment (well under a 1500-byte Ethernet MTU)


class MsgType(IntEnum):
    """Every control message. Names/codes 0-49 mirror the reference PacketType
    (packets.py:9-60; its 6-char binary strings are these integers); >= 64 are new."""

    PING = 0
    ACK = 1
    INTRODUCE = 2
    INTRODUCE_ACK = 3
    FETCH_INTRODUCER = 4
    FETCH_INTRODUCER_ACK = 5
    ELECTION = 6
    COORDINATE = 7
    COORDINATE_ACK = 8
    UPDATE_INTRODUCER = 9
    DOWNLOAD_FILE = 10
    DOWNLOAD_FILE_SUCCESS = 11
    DOWNLOAD_FILE_FAIL = 12
    DELETE_FILE = 13
    DELETE_FILE_ACK = 14
    DELETE_FILE_NAK = 15
    GET_FILE = 16
    GET_FILE_SUCCESS = 17
    GET_FILE_FAIL = 18
    PUT_REQUEST = 19
    LIST_FILE_REQUEST = 20
    LIST_FILE_REQUEST_ACK = 21
    GET_FILE_REQUEST = 22
    GET_FILE_REQUEST_ACK = 23
    PUT_REQUEST_ACK = 24
    PUT_REQUEST_SUCCESS = 25
    DELETE_FILE_REQUEST = 26
    DELETE_FILE_REQUEST_ACK = 27
    DELETE_FILE_REQUEST_SUCCESS = 28
    DELETE_FILE_REQUEST_FAIL = 29
    PUT_REQUEST_FAIL = 30
    REPLICATE_FILE = 31
    REPLICATE_FILE_SUCCESS = 32
    REPLICATE_FILE_FAIL = 33
    ALL_LOCAL_FILES = 34
    GET_FILE_NAMES_REQUEST = 35
    GET_FILE_NAMES_REQUEST_ACK = 36
    SUBMIT_JOB_REQUEST = 37
    SUBMIT_JOB_REQUEST_ACK = 38
    WORKER_TASK_REQUEST = 39
    WORKER_TASK_REQUEST_ACK = 40
    SUBMIT_JOB_REQUEST_SUCCESS = 41
    WORKER_KILL_TASK_REQUEST = 42
    WORKER_KILL_TASK_REQUEST_ACK = 43
    SUBMIT_JOB_RELAY = 44
    WORKER_TASK_ACK_RELAY = 45
    ALL_LOCAL_FILES_RELAY = 46
    SET_BATCH_SIZE = 47
    GET_C2_COMMAND = 48
    GET_C2_COMMAND_ACK = 49
    # ---- new in this framework ----
    PING_REQ = 64            # SWIM indirect probe: "ping X for me"
    PING_REQ_ACK = 65
    ELECTION_OK = 66         # bully: a higher-priority node takes over the election
    LEAVE = 67               # graceful leave (reference menu option 4 just went silent)
    GET_C1_COMMAND = 68
    GET_C1_COMMAND_ACK = 69
    GET_ASSIGNMENTS = 70     # C5 forwarded to the coordinator
    GET_ASSIGNMENTS_ACK = 71
    SET_BATCH_SIZE_ACK = 72
    STANDBY_SYNC = 73        # full coordinator state snapshot to the standby
    JOB_STATUS = 74
    JOB_STATUS_ACK = 75
    PUT_MANY_REQUEST = 76    # one PUT of several files (an output bundle): one leader round trip
    PUT_MANY_REPLY = 77      # {"ok": [names], "failed": [names]}
    DOWNLOAD_MANY = 78       # leader -> replica: pull these (name, version)s from one outbox
    DOWNLOAD_MANY_REPLY = 79  # {"ok": {name: versions}, "failed": [names]}
    FILES_STORED = 80        # writer -> leader: files it stored on their replicas itself (put_many_direct)
    FILES_STORED_ACK = 81
    GET_OUTPUT = 82          # get-output at the coordinator: final_<job>.json from its gathered results
    GET_OUTPUT_ACK = 83      # {"name": store name of the rendered final file, or None}
    ERROR = 127


@dataclass
class Frame:
    type: MsgType
    sender: str
    payload: Dict[str, Any] = field(default_factory=dict)
    seq: int = 0          # request id; replies echo it
    flags: int = 0        # bit0: is_reply

    @property
    def is_reply(self) -> bool:
        return bool(self.flags & 1)


class FrameError(ValueError):
    pass


_msg_counter = int(time.time() * 1000) & 0xFFFFFFFF


def _next_msg_id() -> int:
    global _msg_counter
    _msg_counter = (_msg_counter + 1) & 0xFFFFFFFF
    return _msg_counter


def encode(frame: Frame, mtu_payload: int = MTU_PAYLOAD) -> List[bytes]:
    """Frame -> list of datagrams (one unless the body exceeds one MTU)."""
    sender = frame.sender.encode()
    if len(sender) > 255:
        raise FrameError("sender name too long")
    body = json.dumps(frame.payload, separators=(",", ":"), default=_json_default).encode()
    chunks = [body[i:i + mtu_payload] for i in range(0, len(body), mtu_payload)] or [b""]
    if len(chunks) > 0xFFFF:
        raise FrameError("message too large")
    msg_id = _next_msg_id() if len(chunks) > 1 else 0
    out = []
    for idx, ch in enumerate(chunks):
        hdr = _HDR.pack(MAGIC, VERSION, int(frame.type), frame.flags, frame.seq, idx, len(chunks), msg_id, len(sender))
        out.append(hdr + sender + ch)
    return out


def _json_default(o):
    try:
        import numpy as np

        if isinstance(o, np.integer):
            return int(o)
        if isinstance(o, np.floating):
            return float(o)
        if isinstance(o, np.ndarray):
            return o.tolist()
    except ImportError:  # pragma: no cover
        pass
    if isinstance(o, (set, tuple)):
        return list(o)
    raise TypeError(f"not JSON serialisable: {type(o)}")


def decode_fragment(data: bytes) -> Tuple[int, int, int, Frame, bytes]:
    """datagram -> (msg_id, frag_idx, frag_cnt, frame-with-empty-payload, body chunk)."""
    if len(data) < _HDR.size:
        raise FrameError("short datagram")
    magic, ver, typ, flags, seq, idx, cnt, msg_id, slen = _HDR.unpack_from(data)
    if magic != MAGIC or ver != VERSION:
        raise FrameError("bad magic/version")
    off = _HDR.size
    sender = data[off:off + slen].decode()
    body = data[off + slen:]
    try:
        mtype = MsgType(typ)
    except ValueError as e:
        raise FrameError(f"unknown message type {typ}") from e
    if cnt == 0 or idx >= cnt:
        raise FrameError("bad fragment index")
    return msg_id, idx, cnt, Frame(mtype, sender, {}, seq, flags), body


def decode(data: bytes) -> Frame:
    """Single-datagram decode (raises if the message was fragmented)."""
    msg_id, idx, cnt, fr, body = decode_fragment(data)
    if cnt != 1:
        raise FrameError("fragmented message: use Reassembler")
    fr.payload = _parse(body)
    return fr


def _parse(body: bytes) -> Dict[str, Any]:
    if not body:
        return {}
    try:
        obj = json.loads(body.decode())
    except (UnicodeDecodeError, json.JSONDecodeError) as e:
        raise FrameError(f"bad payload: {e}") from e
    if not isinstance(obj, dict):
        raise FrameError("payload must be an object")
    return obj


class Reassembler:
    """Collects fragments per (sender, msg_id); drops incomplete messages after `ttl` seconds."""

    def __init__(self, ttl: float = 5.0, clock=time.monotonic):
        self.ttl, self.clock = ttl, clock
        self._parts: Dict[Tuple[str, int], Tuple[float, Frame, List[Optional[bytes]]]] = {}

    def feed(self, data: bytes) -> Optional[Frame]:
        msg_id, idx, cnt, fr, body = decode_fragment(data)
        if cnt == 1:
            fr.payload = _parse(body)
            return fr
        key = (fr.sender, msg_id)
        now = self.clock()
        self._gc(now)
        if key not in self._parts:
            self._parts[key] = (now, fr, [None] * cnt)
        _, fr0, parts = self._parts[key]
        if len(parts) != cnt:
            raise FrameError("fragment count mismatch")
        parts[idx] = body
        if all(p is not None for p in parts):
            del self._parts[key]
            fr0.payload = _parse(b"".join(parts))
            return fr0
        return None

    def _gc(self, now: float) -> None:
        dead = [k for k, (t, _, _) in self._parts.items() if now - t > self.ttl]
        for k in dead:
            del self._parts[k]

    def pending(self) -> int:
        return len(self._parts)
