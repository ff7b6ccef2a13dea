"""Minimal RFC 6455 WebSocket client (the simulator's side of the wire) for tests and benches of
pp_serve: handshake with Sec-WebSocket-Key, masked text frames, ping/close."""
import base64
import hashlib
import os
import socket
import struct

GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"


class WSClient:
    def __init__(self, port, host="127.0.0.1", path="/socket.io/?EIO=4&transport=websocket", timeout=30.0):
        self.s = socket.create_connection((host, port), timeout=timeout)
        self.s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        key = base64.b64encode(os.urandom(16))
        self.s.sendall(b"GET " + path.encode() + b" HTTP/1.1\r\nHost: " + host.encode() +
                       b"\r\nUpgrade: websocket\r\nConnection: Upgrade\r\nSec-WebSocket-Key: " + key +
                       b"\r\nSec-WebSocket-Version: 13\r\n\r\n")
        resp = b""
        while b"\r\n\r\n" not in resp:
            chunk = self.s.recv(4096)
            if not chunk:
                raise ConnectionError("closed during handshake")
            resp += chunk
        head, self.buf = resp.split(b"\r\n\r\n", 1)
        self.status_line = head.split(b"\r\n")[0]
        want = base64.b64encode(hashlib.sha1(key + GUID).digest())
        self.accept_ok = b"Sec-WebSocket-Accept: " + want in head

    def send_frame(self, payload, opcode=1, fin=True):
        mask = os.urandom(4)
        n = len(payload)
        hdr = bytes([(0x80 if fin else 0) | opcode])
        if n < 126:
            hdr += bytes([0x80 | n])
        elif n < 65536:
            hdr += bytes([0x80 | 126]) + struct.pack(">H", n)
        else:
            hdr += bytes([0x80 | 127]) + struct.pack(">Q", n)
        body = bytes(b ^ mask[i & 3] for i, b in enumerate(payload))
        self.s.sendall(hdr + mask + body)

    def send(self, text):
        self.send_frame(text if isinstance(text, bytes) else text.encode())

    def _need(self, n):
        while len(self.buf) < n:
            chunk = self.s.recv(1 << 16)
            if not chunk:
                raise ConnectionError("closed")
            self.buf += chunk

    def recv_frame(self):
        self._need(2)
        b0, b1 = self.buf[0], self.buf[1]
        n, h = b1 & 0x7F, 2
        if n == 126:
            self._need(4)
            n, h = struct.unpack(">H", self.buf[2:4])[0], 4
        elif n == 127:
            self._need(10)
            n, h = struct.unpack(">Q", self.buf[2:10])[0], 10
        self._need(h + n)
        payload = self.buf[h:h + n]
        self.buf = self.buf[h + n:]
        return b0 & 0x0F, payload

    def recv(self):
        """Next text message (answers pings on the way)."""
        while True:
            op, p = self.recv_frame()
            if op == 1:
                return p
            if op == 8:
                raise ConnectionError("server closed")

    def close(self):
        try:
            self.send_frame(struct.pack(">H", 1000), opcode=8)
            self.recv_frame()
        except OSError:
            pass
        self.s.close()
