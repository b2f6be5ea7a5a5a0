"""AES-256-CBC for secret config values (reference ``core/_private/crypto.py`` AESCipher +
``utils.py:3412-3490`` privacy handling).

The reference relies on pycryptodome, which is not available here; this is a compact,
dependency-free AES (FIPS-197) with PKCS#7 padding.  Wire format is unchanged:
``base64(iv || ciphertext)``, and encrypted config values carry the ``[AES]:`` prefix.
Only small strings (credentials in configs) go through it, so a table-driven pure-Python
block cipher is adequate.
"""
from __future__ import annotations

import base64
import collections.abc
import copy
import os
from typing import Any, Dict

ENCRYPTION_PREFIX = "[AES]:"
PRIVACY_CONFIG_KEYS = ["credentials", "secret", "password", ".key", "_key"]
PRIVACY_REPLACEMENT = "VALUE-PROTECTED"
PRIVACY_REPLACEMENT_TEMPLATE = "VALUE-{}PROTECTED"
# default config secret (hex, 32 bytes); override with CLOUDTIK_CONFIG_SECRET
_DEFAULT_SECRET = "5fd0c5e4a2b3617e9d8c4b2a1f0e9d8c7b6a59483726150f1e2d3c4b5a697887"


def _xtime(a):
    return ((a << 1) ^ 0x1B) & 0xFF if a & 0x80 else a << 1


def _build_tables():
    sbox = [0] * 256
    inv = [0] * 256
    p = q = 1
    while True:
        p = p ^ _xtime(p)                    # multiply p by 3
        q ^= q << 1
        q ^= q << 2
        q ^= q << 4
        q &= 0xFF
        if q & 0x80:
            q ^= 0x09                        # divide q by 3
        x = q ^ ((q << 1) | (q >> 7)) ^ ((q << 2) | (q >> 6)) ^ ((q << 3) | (q >> 5)) ^ ((q << 4) | (q >> 4))
        x = (x ^ 0x63) & 0xFF
        sbox[p] = x
        inv[x] = p
        if p == 1:
            break
    sbox[0] = 0x63
    inv[0x63] = 0
    return sbox, inv


_SBOX, _INV_SBOX = _build_tables()


def _mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = _xtime(a)
        b >>= 1
    return r


def _expand_key(key: bytes):
    nk = len(key) // 4
    nr = nk + 6
    w = [list(key[4 * i:4 * i + 4]) for i in range(nk)]
    rcon = 1
    for i in range(nk, 4 * (nr + 1)):
        t = list(w[i - 1])
        if i % nk == 0:
            t = t[1:] + t[:1]
            t = [_SBOX[b] for b in t]
            t[0] ^= rcon
            rcon = _xtime(rcon)
        elif nk > 6 and i % nk == 4:
            t = [_SBOX[b] for b in t]
        w.append([a ^ b for a, b in zip(w[i - nk], t)])
    return [sum(w[4 * r:4 * r + 4], []) for r in range(nr + 1)]


def _encrypt_block(rk, block):
    s = [b ^ k for b, k in zip(block, rk[0])]
    nr = len(rk) - 1
    for r in range(1, nr + 1):
        s = [_SBOX[b] for b in s]
        s = [s[(i + 4 * (i % 4)) % 16] for i in range(16)]  # ShiftRows (column-major state)
        if r != nr:
            t = []
            for c in range(4):
                a = s[4 * c:4 * c + 4]
                t += [_mul(a[0], 2) ^ _mul(a[1], 3) ^ a[2] ^ a[3],
                      a[0] ^ _mul(a[1], 2) ^ _mul(a[2], 3) ^ a[3],
                      a[0] ^ a[1] ^ _mul(a[2], 2) ^ _mul(a[3], 3),
                      _mul(a[0], 3) ^ a[1] ^ a[2] ^ _mul(a[3], 2)]
            s = t
        s = [b ^ k for b, k in zip(s, rk[r])]
    return bytes(s)


def _decrypt_block(rk, block):
    nr = len(rk) - 1
    s = [b ^ k for b, k in zip(block, rk[nr])]
    for r in range(nr - 1, -1, -1):
        s = [s[(i - 4 * (i % 4)) % 16] for i in range(16)]  # InvShiftRows
        s = [_INV_SBOX[b] for b in s]
        s = [b ^ k for b, k in zip(s, rk[r])]
        if r != 0:
            t = []
            for c in range(4):
                a = s[4 * c:4 * c + 4]
                t += [_mul(a[0], 14) ^ _mul(a[1], 11) ^ _mul(a[2], 13) ^ _mul(a[3], 9),
                      _mul(a[0], 9) ^ _mul(a[1], 14) ^ _mul(a[2], 11) ^ _mul(a[3], 13),
                      _mul(a[0], 13) ^ _mul(a[1], 9) ^ _mul(a[2], 14) ^ _mul(a[3], 11),
                      _mul(a[0], 11) ^ _mul(a[1], 13) ^ _mul(a[2], 9) ^ _mul(a[3], 14)]
            s = t
    return bytes(s)


class AESCipher:
    block_size = 16

    def __init__(self, key: bytes):
        if len(key) not in (16, 24, 32):
            raise ValueError("AES key must be 16, 24 or 32 bytes")
        self.key = key
        self._rk = _expand_key(key)

    def encrypt_block(self, b: bytes) -> bytes:
        return _encrypt_block(self._rk, b)

    def decrypt_block(self, b: bytes) -> bytes:
        return _decrypt_block(self._rk, b)

    def encrypt(self, raw: str, iv: bytes = None) -> bytes:
        data = raw.encode("utf-8")
        pad = 16 - len(data) % 16
        data += bytes([pad]) * pad
        iv = iv or os.urandom(16)
        prev, out = iv, [iv]
        for i in range(0, len(data), 16):
            blk = bytes(a ^ b for a, b in zip(data[i:i + 16], prev))
            prev = self.encrypt_block(blk)
            out.append(prev)
        return base64.b64encode(b"".join(out))

    def decrypt(self, enc: bytes) -> str:
        raw = base64.b64decode(enc)
        iv, ct = raw[:16], raw[16:]
        prev, out = iv, []
        for i in range(0, len(ct), 16):
            blk = ct[i:i + 16]
            out.append(bytes(a ^ b for a, b in zip(self.decrypt_block(blk), prev)))
            prev = blk
        data = b"".join(out)
        return data[:-data[-1]].decode("utf-8") if data else ""

    @staticmethod
    def generate_key() -> bytes:
        return os.urandom(32)


def get_config_cipher() -> AESCipher:
    return AESCipher(bytes.fromhex(os.environ.get("CLOUDTIK_CONFIG_SECRET", _DEFAULT_SECRET)))


def is_config_key_with_privacy(key) -> bool:
    if not isinstance(key, str):
        return False
    k = key.lower()
    return any(w in k for w in PRIVACY_CONFIG_KEYS)


def _hide(v, _):
    if not isinstance(v, str):
        return v
    n, r = len(v), len(PRIVACY_REPLACEMENT)
    return PRIVACY_REPLACEMENT_TEMPLATE.format("-" * (n - r)) if n > r else PRIVACY_REPLACEMENT


def process_config_with_privacy(config, func=_hide, param=None):
    if isinstance(config, collections.abc.Mapping):
        for k, v in config.items():
            if isinstance(v, (collections.abc.Mapping, list)):
                process_config_with_privacy(v, func, param)
            elif is_config_key_with_privacy(k):
                config[k] = func(v, param)
    elif isinstance(config, list):
        for item in config:
            if isinstance(item, (collections.abc.Mapping, list)):
                process_config_with_privacy(item, func, param)


def _enc(v, cipher):
    if not isinstance(v, str) or v.startswith(ENCRYPTION_PREFIX):
        return v
    return ENCRYPTION_PREFIX + cipher.encrypt(v).decode("utf-8")


def _dec(v, cipher):
    if not isinstance(v, str) or not v.startswith(ENCRYPTION_PREFIX):
        return v
    return cipher.decrypt(v[len(ENCRYPTION_PREFIX):].encode("utf-8"))


def encrypt_config(config: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(config)
    process_config_with_privacy(out, _enc, get_config_cipher())
    return out


def decrypt_config(config: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(config)
    process_config_with_privacy(out, _dec, get_config_cipher())
    return out


def with_privacy(config: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(config)
    process_config_with_privacy(out)
    return out


def encrypt_string(v: str) -> str:
    return get_config_cipher().encrypt(v).decode("utf-8") if v is not None else v


def decrypt_string(v: str) -> str:
    return get_config_cipher().decrypt(v.encode("utf-8")) if v is not None else v
