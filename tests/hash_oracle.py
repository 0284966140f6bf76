"""Python restatement of sg_hash64 / part_of (swarm_amd/csrc/sg_abi.hip) — test oracle."""
M = (1 << 64) - 1


def mix64(x):
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & M
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & M
    x ^= x >> 33
    return x


def hash64(rec: bytes) -> int:
    n = len(rec)
    h = 0x9E3779B97F4A7C15 ^ ((n * 0xFF51AFD7ED558CCD) & M)
    for o in range(0, n, 8):
        w = int.from_bytes(rec[o:o + 8], "little")
        h = ((h ^ mix64(w)) * 0x9FB21C651E98DF25) & M
        h ^= h >> 29
    return mix64(h)


def part_of(h: int, parts: int) -> int:
    return ((h >> 32) * parts) >> 32
