"""Minimal RESP2 client for the native state server (``cloudtik-state-server``).

Replaces the reference's dependency on the ``redis`` python package
(core/_private/state/redis_shards_client.py:36-140).  Thread-safe for request/response use
(one lock per connection); a :class:`PubSub` owns its own connection.
"""
from __future__ import annotations

import socket
import threading
import time
from typing import Any, Iterable, List, Optional, Tuple, Union

Bytes = Union[bytes, str, int, float]


class RespError(Exception):
    pass


def _enc(v: Bytes) -> bytes:
    if isinstance(v, bytes):
        return v
    if isinstance(v, str):
        return v.encode()
    return str(v).encode()


def encode_command(*args: Bytes) -> bytes:
    parts = [b"*%d\r\n" % len(args)]
    for a in args:
        b = _enc(a)
        parts.append(b"$%d\r\n" % len(b))
        parts.append(b)
        parts.append(b"\r\n")
    return b"".join(parts)


class _Reader:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = bytearray()

    def _fill(self):
        chunk = self.sock.recv(65536)
        if not chunk:
            raise ConnectionError("state server closed the connection")
        self.buf += chunk

    def _line(self) -> bytes:
        while True:
            i = self.buf.find(b"\r\n")
            if i >= 0:
                line = bytes(self.buf[:i])
                del self.buf[:i + 2]
                return line
            self._fill()

    def _exact(self, n: int) -> bytes:
        while len(self.buf) < n + 2:
            self._fill()
        out = bytes(self.buf[:n])
        del self.buf[:n + 2]
        return out

    def read(self) -> Any:
        line = self._line()
        t, rest = line[:1], line[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            raise RespError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else self._exact(n)
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [self.read() for _ in range(n)]
        raise RespError(f"bad RESP type byte {t!r}")


class RespConnection:
    def __init__(self, host: str = "127.0.0.1", port: int = 6789, password: Optional[str] = None,
                 timeout: Optional[float] = 10.0, connect_retries: int = 20,
                 client_name: Optional[str] = None):
        self.host, self.port, self.password = host, int(port), password
        self.timeout = timeout
        self.connect_retries = connect_retries
        self.client_name = client_name
        self._lock = threading.RLock()
        self._sock: Optional[socket.socket] = None
        self._reader: Optional[_Reader] = None

    # ------------------------------------------------------------------ connection
    def connect(self):
        last = None
        for i in range(max(1, self.connect_retries)):
            try:
                s = socket.create_connection((self.host, self.port), timeout=self.timeout)
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                self._sock, self._reader = s, _Reader(s)
                if self.password:
                    self._roundtrip(("AUTH", self.password))
                if self.client_name:
                    self._roundtrip(("CLIENT", "SETNAME", self.client_name))
                return self
            except (ConnectionError, OSError) as e:
                last = e
                self.close()
                time.sleep(min(0.05 * (2 ** i), 1.0))
        raise ConnectionError(f"cannot connect to state server {self.host}:{self.port}: {last}")

    def close(self):
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
        self._sock, self._reader = None, None

    def _roundtrip(self, args: Tuple[Bytes, ...]):
        self._sock.sendall(encode_command(*args))
        return self._reader.read()

    def execute(self, *args: Bytes):
        with self._lock:
            for attempt in range(2):
                if self._sock is None:
                    self.connect()
                try:
                    return self._roundtrip(args)
                except (ConnectionError, OSError):
                    self.close()
                    if attempt:
                        raise

    def pipeline(self, commands: Iterable[Tuple[Bytes, ...]]) -> List[Any]:
        """Send all commands in one write and read all replies (errors are returned)."""
        commands = list(commands)
        with self._lock:
            if self._sock is None:
                self.connect()
            self._sock.sendall(b"".join(encode_command(*c) for c in commands))
            out = []
            for _ in commands:
                try:
                    out.append(self._reader.read())
                except RespError as e:
                    out.append(e)
            return out

    # ------------------------------------------------------------------ convenience API
    def ping(self) -> bool:
        return self.execute("PING") == "PONG"

    def get(self, key) -> Optional[bytes]:
        return self.execute("GET", key)

    def set(self, key, value, nx: bool = False, ex: Optional[int] = None) -> bool:
        args: List[Bytes] = ["SET", key, value]
        if nx:
            args.append("NX")
        if ex is not None:
            args += ["EX", int(ex)]
        return self.execute(*args) == "OK"

    def delete(self, *keys) -> int:
        return self.execute("DEL", *keys)

    def exists(self, *keys) -> int:
        return self.execute("EXISTS", *keys)

    def keys(self, pattern="*") -> List[bytes]:
        return self.execute("KEYS", pattern)

    def incr(self, key, by: int = 1) -> int:
        return self.execute("INCRBY", key, by)

    def hset(self, key, field, value) -> int:
        return self.execute("HSET", key, field, value)

    def hget(self, key, field) -> Optional[bytes]:
        return self.execute("HGET", key, field)

    def hdel(self, key, *fields) -> int:
        return self.execute("HDEL", key, *fields)

    def hgetall(self, key) -> dict:
        flat = self.execute("HGETALL", key) or []
        return {flat[i]: flat[i + 1] for i in range(0, len(flat), 2)}

    def rpush(self, key, *values) -> int:
        return self.execute("RPUSH", key, *values)

    def lrange(self, key, start=0, end=-1) -> List[bytes]:
        return self.execute("LRANGE", key, start, end)

    def ltrim(self, key, start, end):
        return self.execute("LTRIM", key, start, end)

    def publish(self, channel, message) -> int:
        return self.execute("PUBLISH", channel, message)

    def save(self):
        return self.execute("SAVE")

    def config_get(self, pattern) -> dict:
        flat = self.execute("CONFIG", "GET", pattern) or []
        return {flat[i].decode(): flat[i + 1].decode() for i in range(0, len(flat), 2)}

    def config_set(self, name, value):
        return self.execute("CONFIG", "SET", name, value)

    def pubsub(self) -> "PubSub":
        return PubSub(self.host, self.port, self.password, self.timeout)


class PubSub:
    """Subscriber connection: ``subscribe(ch)``, then ``get_message(timeout)``."""

    def __init__(self, host, port, password=None, timeout=None):
        self.conn = RespConnection(host, port, password, timeout=timeout).connect()
        self.conn._sock.settimeout(None)

    def subscribe(self, *channels):
        self.conn._sock.sendall(encode_command("SUBSCRIBE", *channels))
        for _ in channels:
            self.conn._reader.read()

    def psubscribe(self, *patterns):
        self.conn._sock.sendall(encode_command("PSUBSCRIBE", *patterns))
        for _ in patterns:
            self.conn._reader.read()

    def get_message(self, timeout: Optional[float] = 1.0):
        """Returns ``(channel, data)`` or ``None`` on timeout."""
        sock = self.conn._sock
        if not self.conn._reader.buf:
            sock.settimeout(timeout)
            try:
                self.conn._reader._fill()
            except socket.timeout:
                return None
            finally:
                sock.settimeout(None)
        msg = self.conn._reader.read()
        if msg[0] == b"message":
            return msg[1], msg[2]
        if msg[0] == b"pmessage":
            return msg[2], msg[3]
        return None

    def close(self):
        self.conn.close()
