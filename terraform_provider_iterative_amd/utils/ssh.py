"""SSH key material (references: ``iterative/utils/ssh.go`` and
``task/common/ssh/deterministic_key_pair_ssh.go``).

* :func:`private_pem` — random RSA-4096 key, PKCS#1 PEM (``ssh-keygen`` when present, else
  the pure-Python generator below).
* :func:`public_from_private_pem` — ``ssh-rsa AAAA...`` authorized_keys line.
* :class:`DeterministicSSHKeyPair` — RSA key derived from ``(secret, realm)``: the same inputs
  always give the same key (the reference uses cloudflare/gokey for this; the derivation here
  is our own HMAC-DRBG construction, so keys are stable across runs of this framework but
  not equal to gokey's).
* :func:`run_command` — run a command over SSH with the system ``ssh`` client.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import secrets
import shutil
import subprocess
import tempfile
from typing import Callable, Optional, Tuple

_SMALL_PRIMES = []
_sieve = bytearray([1]) * 20000
for _i in range(2, 20000):
    if _sieve[_i]:
        _SMALL_PRIMES.append(_i)
        _sieve[_i * _i::_i] = bytearray(len(_sieve[_i * _i::_i]))
del _sieve


class HmacDrbg:
    """NIST SP 800-90A HMAC_DRBG (SHA-256), used as a deterministic randomness source."""

    def __init__(self, seed: bytes):
        self.k = b"\x00" * 32
        self.v = b"\x01" * 32
        self._update(seed)

    def _update(self, data: bytes = b"") -> None:
        self.k = hmac.new(self.k, self.v + b"\x00" + data, hashlib.sha256).digest()
        self.v = hmac.new(self.k, self.v, hashlib.sha256).digest()
        if data:
            self.k = hmac.new(self.k, self.v + b"\x01" + data, hashlib.sha256).digest()
            self.v = hmac.new(self.k, self.v, hashlib.sha256).digest()

    def generate(self, n: int) -> bytes:
        out = b""
        while len(out) < n:
            self.v = hmac.new(self.k, self.v, hashlib.sha256).digest()
            out += self.v
        self._update()
        return out[:n]


def _is_probable_prime(n: int, rand: Callable[[int], bytes], rounds: int = 40) -> bool:
    if n < 2:
        return False
    for p in _SMALL_PRIMES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    nbytes = (n.bit_length() + 7) // 8
    for _ in range(rounds):
        a = 2 + int.from_bytes(rand(nbytes), "big") % (n - 3)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = pow(x, 2, n)
            if x == n - 1:
                break
        else:
            return False
    return True


def _random_prime(bits: int, rand: Callable[[int], bytes], e: int = 65537) -> int:
    while True:
        candidate = int.from_bytes(rand(bits // 8), "big")
        candidate |= (1 << (bits - 1)) | (1 << (bits - 2)) | 1  # top two bits: n has 2*bits
        if candidate % e == 1:
            continue
        if _is_probable_prime(candidate, rand):
            return candidate


def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    raw = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(raw)]) + raw


def _der_int(v: int) -> bytes:
    raw = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")
    return b"\x02" + _der_len(len(raw)) + raw


def _der_seq(*items: bytes) -> bytes:
    body = b"".join(items)
    return b"\x30" + _der_len(len(body)) + body


def _parse_der_ints(data: bytes):
    """Integers of a DER SEQUENCE (enough to read PKCS#1 RSAPrivateKey)."""
    def read_len(buf, i):
        first = buf[i]
        if first < 0x80:
            return first, i + 1
        n = first & 0x7F
        return int.from_bytes(buf[i + 1:i + 1 + n], "big"), i + 1 + n

    if data[0] != 0x30:
        raise ValueError("not a DER sequence")
    _, i = read_len(data, 1)
    out = []
    while i < len(data):
        if data[i] != 0x02:
            raise ValueError("unexpected DER tag")
        length, i = read_len(data, i + 1)
        out.append(int.from_bytes(data[i:i + length], "big"))
        i += length
    return out


class RSAKey:
    def __init__(self, n: int, e: int, d: int, p: int, q: int):
        self.n, self.e, self.d, self.p, self.q = n, e, d, p, q

    @classmethod
    def generate(cls, bits: int = 4096, rand: Optional[Callable[[int], bytes]] = None) -> "RSAKey":
        rand = rand or secrets.token_bytes
        e = 65537
        while True:
            p = _random_prime(bits // 2, rand)
            q = _random_prime(bits // 2, rand)
            if p == q:
                continue
            if p < q:
                p, q = q, p
            phi = (p - 1) * (q - 1)
            try:
                d = pow(e, -1, phi)
            except ValueError:
                continue
            return cls(p * q, e, d, p, q)

    def private_pem(self) -> str:
        der = _der_seq(_der_int(0), _der_int(self.n), _der_int(self.e), _der_int(self.d),
                       _der_int(self.p), _der_int(self.q), _der_int(self.d % (self.p - 1)),
                       _der_int(self.d % (self.q - 1)), _der_int(pow(self.q, -1, self.p)))
        b64 = base64.b64encode(der).decode()
        lines = [b64[i:i + 64] for i in range(0, len(b64), 64)]
        return "-----BEGIN RSA PRIVATE KEY-----\n%s\n-----END RSA PRIVATE KEY-----\n" % "\n".join(lines)

    @classmethod
    def from_pem(cls, pem: str) -> "RSAKey":
        body = "".join(l for l in pem.strip().splitlines() if not l.startswith("-----"))
        ints = _parse_der_ints(base64.b64decode(body))
        return cls(ints[1], ints[2], ints[3], ints[4], ints[5])

    def public_openssh(self) -> str:
        def mpint(v: int) -> bytes:
            raw = v.to_bytes((v.bit_length() + 8) // 8, "big")
            return len(raw).to_bytes(4, "big") + raw

        blob = len(b"ssh-rsa").to_bytes(4, "big") + b"ssh-rsa" + mpint(self.e) + mpint(self.n)
        return "ssh-rsa " + base64.b64encode(blob).decode() + "\n"


def private_pem(bits: int = 4096) -> str:
    """Random RSA private key (PKCS#1 PEM)."""
    keygen = shutil.which("ssh-keygen")
    if keygen:
        with tempfile.TemporaryDirectory() as tmp:
            path = os.path.join(tmp, "id")
            result = subprocess.run([keygen, "-q", "-t", "rsa", "-b", str(bits), "-m", "PEM",
                                     "-N", "", "-f", path], capture_output=True)
            if result.returncode == 0:
                with open(path) as handle:
                    return handle.read()
    return RSAKey.generate(bits).private_pem()


def public_from_private_pem(pem: str) -> str:
    return RSAKey.from_pem(pem).public_openssh()


class DeterministicSSHKeyPair:
    """RSA key pair derived from ``(key, realm)`` (``NewDeterministicSSHKeyPair``)."""

    def __init__(self, key: str, realm: str, bits: int = 4096):
        seed = hashlib.pbkdf2_hmac("sha256", key.encode(), ("tpi-ssh:" + realm).encode(),
                                   4096, 64)
        self._key = RSAKey.generate(bits, HmacDrbg(seed).generate)

    def private_string(self) -> str:
        return self._key.private_pem()

    def public_string(self) -> str:
        return self._key.public_openssh()


def run_command(command: str, timeout: float, address: str, user: str,
                private_key: str) -> Tuple[str, int]:
    """Run ``command`` on ``user@address`` (host key not checked, like the reference)."""
    host, _, port = address.rpartition(":")
    with tempfile.NamedTemporaryFile("w", delete=False) as handle:
        handle.write(private_key)
        key_path = handle.name
    os.chmod(key_path, 0o600)
    try:
        result = subprocess.run(
            ["ssh", "-i", key_path, "-p", port or "22", "-o", "StrictHostKeyChecking=no",
             "-o", "UserKnownHostsFile=/dev/null", "-o", "ConnectTimeout=%d" % max(1, int(timeout)),
             "%s@%s" % (user, host or address), command],
            capture_output=True, text=True, timeout=timeout + 30)
        return result.stdout + result.stderr, result.returncode
    finally:
        os.unlink(key_path)
