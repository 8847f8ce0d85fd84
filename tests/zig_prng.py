"""Restatement of Zig 0.11 std.rand.Xoshiro256 (+ SplitMix64 seeding) and
Xoshiro256.fill — needed to reproduce the reference's "checksum stability"
known-answer test (src/vsr/checksum.zig:172-181, `std.rand.Xoshiro256.init(92)`).
Zig std is third-party to the reference (pinned by scripts/install_zig.sh:4);
this restatement is accepted only because the stability hash matches."""

M64 = (1 << 64) - 1


def _rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & M64


class SplitMix64:
    def __init__(self, seed):
        self.s = seed & M64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)


class Xoshiro256:
    def __init__(self, seed):
        g = SplitMix64(seed)
        self.s = [g.next(), g.next(), g.next(), g.next()]

    def next(self):
        s = self.s
        r = (_rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 45)
        return r

    def fill(self, n):
        """Zig Xoshiro256.fill: 8 bytes LE per next(); a final partial word."""
        out = bytearray()
        full = n - (n & 7)
        while len(out) < full:
            out += self.next().to_bytes(8, "little")
        if len(out) != n:
            out += self.next().to_bytes(8, "little")[: n - len(out)]
        return bytes(out)


def stability_messages():
    """The 896 messages of checksum.zig:146-181, in order."""
    msgs = []
    for sub in range(128):  # zeros of various lengths
        msgs.append(bytes(sub))
    for sub in range(64 * 8):  # 64 bytes with exactly one bit set
        m = bytearray(64)
        m[sub // 8] = 1 << (sub % 8)
        msgs.append(bytes(m))
    prng = Xoshiro256(92)
    for sub in range(256):  # pseudo-random data of various lengths
        msgs.append(prng.fill(sub + 13))
    return msgs


STABILITY_HASH = 0x82DCAACF4875B279446825B6830D1263  # checksum.zig:194
