"""The CRC-16 arithmetic the decode kernels use instead of tables (round 6), restated in Python
and checked against the oracle's bit-serial CRC-16 (oracle/flac_oracle.c, libFLAC's
FLAC__crc16 @ read_frame_'s footer check, LibFlac.dll@0x10011a01).

- The decode tails' zero test (bnflac_kernels.hip st_crc16_ok / crcz_w / crcz_zero): the CRC of
  frame + footer is zero iff the message has even parity and is 0 mod T = x^15 + x + 1
  (P = x^16 + x^15 + x^2 + 1 = (x + 1) T), with the remainder kept mod T^4 = x^60 + x^4 + 1 in
  two words, five operations per 32-bit word.
- k_parse's prefix (crcp_fold / crcp_z): 64-byte lines folded at once mod Q(y) = y^15 + y + 1,
  y = x^32, on little-endian words, byte-swapped once at the end and reduced to the T^4 form.
- The hand-off: the prefix of the lines before some line continued by the tail over the rest
  (st_crc16_ok's `from`), bytes before the frame's first byte cleared.
CPU only: these are the formulas, not the kernels (the GPU tests check the kernels)."""
import random

import pytest

import oracle

M32 = 0xFFFFFFFF
T = (1 << 15) | 3


def bswap(w):
    return int.from_bytes(w.to_bytes(4, "little"), "big")


def crcz_w(z, le):
    """bnflac_kernels.hip crcz_w: one little-endian stream word into the T^4 remainder."""
    r0, r1, px = z
    w = bswap(le)
    h = ((r1 << 32 | r0) >> 28) & M32  # v_alignbit(r1, r0, 28)
    n0 = w ^ h ^ ((h << 4) & M32)
    return (n0, (r0 ^ (h >> 28)) & M32, px)


def crcz_zero(z):
    """crcz_zero: even parity and the 60-bit remainder 0 mod T."""
    r0, r1, px = z
    if bin(px).count("1") & 1:
        return False
    v = ((r1 & 0x0FFFFFFF) << 32) | r0
    for _ in range(4):
        h = v >> 15
        v = (v & 0x7FFF) ^ h ^ (h << 1)
    return v == 0


def words_le(buf):
    return [int.from_bytes(buf[i:i + 4], "little") for i in range(0, len(buf), 4)]


def tail_zero_test(data, b0, b1, z=(0, 0, 0), frm=0):
    """st_crc16_ok over [b0, b1) of `data`, continuing z, which holds the lines [b0 & ~63, frm):
    whole 16-byte blocks from max(b0 & ~63, frm), bytes outside [b0, b1) cleared."""
    p = max(b0 & ~63, frm)
    buf = bytearray(data[p:(b1 + 15) & ~15].ljust(((b1 + 15) & ~15) - p, b"\0"))
    for i in range(len(buf)):
        if p + i < b0 or p + i >= b1:
            buf[i] = 0
    r0, r1, px = z
    for w in words_le(bytes(buf)):
        px ^= w
        r0, r1, _ = crcz_w((r0, r1, 0), w)
    return crcz_zero((r0, r1, px))


def crcp_fold(s, px, line):
    """crcp_fold: one 64-byte line (16 little-endian words) into the mod-Q state."""
    w = words_le(line)
    for x in w:
        px ^= x
    r = [0] * 15
    r[0] = s[13] ^ s[14] ^ w[15] ^ w[0]
    r[1] = s[0] ^ s[13] ^ w[14] ^ w[0]
    r[2] = s[0] ^ s[1] ^ s[14] ^ w[13]
    for d in range(3, 15):
        r[d] = s[d - 2] ^ s[d - 1] ^ w[15 - d]
    return r, px


def crcp_z(s, px):
    """crcp_z: the mod-Q state in the T^4 form (Horner over the byte-swapped words)."""
    z = (0, 0, 0)
    for k in range(14, -1, -1):
        z = crcz_w(z, s[k])
    return (z[0], z[1], px)


def frame_with_footer(rng, n, good=True):
    body = bytes(rng.getrandbits(8) for _ in range(n))
    c = oracle.crc16(body)
    if not good:
        c ^= 1 << rng.randrange(16)
    return body + c.to_bytes(2, "big")


@pytest.mark.parametrize("seed", range(4))
def test_tail_zero_test_matches_crc16(seed):
    rng = random.Random(seed)
    for _ in range(40):
        lead = rng.randrange(0, 130)
        n = rng.randrange(1, 700)
        good = rng.random() < 0.6
        fr = frame_with_footer(rng, n, good)
        data = bytes(rng.getrandbits(8) for _ in range(lead)) + fr + bytes(rng.getrandbits(8) for _ in range(40))
        assert tail_zero_test(data, lead, lead + len(fr)) == good, (lead, n, good)


@pytest.mark.parametrize("seed", range(4))
def test_prefix_handoff_matches_crc16(seed):
    """k_parse's prefix over the frame's first line (masked) and whole lines after it, continued
    by the tail from the prefix's end: the same verdict as the CRC of frame + footer."""
    rng = random.Random(100 + seed)
    for _ in range(30):
        lead = rng.randrange(0, 64 * 3)
        n = rng.randrange(200, 1500)
        good = rng.random() < 0.6
        fr = frame_with_footer(rng, n, good)
        data = bytes(rng.getrandbits(8) for _ in range(lead)) + fr + bytes(rng.getrandbits(8) for _ in range(70))
        b0, b1 = lead, lead + len(fr)
        l0 = b0 >> 6
        nlines = rng.randrange(1, (b1 >> 6) - l0 + 1)  # lines [l0, l0 + nlines) folded, within the frame's reach
        s, px = [0] * 15, 0
        for L in range(l0, l0 + nlines):
            line = bytearray(data[64 * L:64 * L + 64].ljust(64, b"\0"))
            if L == l0:
                for i in range(b0 & 63):
                    line[i] = 0
            s, px = crcp_fold(s, px, bytes(line))
        z = crcp_z(s, px)
        frm = 64 * (l0 + nlines)
        assert frm <= b1
        assert tail_zero_test(data, b0, b1, (z[0], z[1] & 0x0FFFFFFF, bin(z[2]).count("1") & 1), frm) == good


def test_mod_q_state_is_the_remainder_mod_t():
    """The mod-Q state, byte-swapped, is congruent mod T to the lines' polynomial."""
    rng = random.Random(7)

    def pmod(a, m):
        d = m.bit_length() - 1
        while a and a.bit_length() - 1 >= d:
            a ^= m << (a.bit_length() - 1 - d)
        return a

    for _ in range(50):
        n = rng.randrange(1, 8)
        data = bytes(rng.getrandbits(8) for _ in range(64 * n))
        s, px = [0] * 15, 0
        for L in range(n):
            s, px = crcp_fold(s, px, data[64 * L:64 * L + 64])
        v = 0
        for k in range(14, -1, -1):
            v = (v << 32) ^ bswap(s[k])
        m = int.from_bytes(data, "big")
        assert pmod(v, T) == pmod(m, T)
        assert (bin(px).count("1") & 1) == (bin(m).count("1") & 1)
