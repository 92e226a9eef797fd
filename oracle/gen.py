"""numpy restatement of the device tuple generator (vpp_amd/csrc/device.hip k_gen) for the
pool/uniform modes (no "inside a rule" sampling). TEST INFRASTRUCTURE ONLY: lets the CPU
regenerate any shard [index_base, index_base + n) of a device-generated workload, so a
multi-rank run can be checked without moving tuples (tests/test_multirank.py,
tests/test_gpu_parity.py).
"""
import numpy as np

M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _rnd(seed, i, f):
    with np.errstate(over="ignore"):
        return _mix64(np.uint64(seed) ^ _mix64(i * np.uint64(16) + np.uint64(f)))


def gen_tuples(n, seed, index_base=0, ip_pool=None, pool_pct=0, dst_pool_pct=0, port_pool=None, port_pool_pct=0,
               tcp_pct=45, udp_pct=45, nomatch_pct=0, table_id=-1, inside_pct=0, **_):
    if table_id >= 0 and inside_pct > 0:
        raise NotImplementedError("inside-a-rule sampling needs the compiled rules (device only)")
    i = np.arange(index_base, index_base + n, dtype=np.uint64)
    lo = lambda x: (x & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    hi = lambda x: (x >> np.uint64(32)).astype(np.uint64)
    r0, r1, r2, r3, r4, r5 = (_rnd(seed, i, f) for f in range(6))
    pct = lo(r0) % np.uint64(100)
    pp = lo(r3) % np.uint64(100)
    proto = np.where(pp < tcp_pct, 0, np.where(pp < tcp_pct + udp_pct, 1, 2)).astype(np.uint8)
    dp = (r4 & np.uint64(0xFFFF)).astype(np.uint32)
    if port_pool is not None and len(port_pool):
        pool = np.asarray(port_pool, np.uint32)
        use = hi(r4) % np.uint64(100) < port_pool_pct
        dp = np.where(use, pool[(lo(r4) % np.uint64(len(pool))).astype(np.int64)], dp)
    src = lo(r1).astype(np.uint32)
    dst = lo(r2).astype(np.uint32)
    if ip_pool is not None and len(ip_pool):
        pool = np.asarray(ip_pool, np.uint32)
        k = np.uint64(len(pool))
        src = np.where(hi(r1) % np.uint64(100) < pool_pct, pool[(lo(r1) % k).astype(np.int64)], src)
        dst = np.where(hi(r2) % np.uint64(100) < dst_pool_pct, pool[(lo(r2) % k).astype(np.int64)], dst)
    if nomatch_pct:
        src = np.where(pct >= 100 - nomatch_pct, np.uint32(0xF0000000) | (lo(r1).astype(np.uint32) & np.uint32(0x0FFFFFFF)),
                       src)
    sport = (r5 & np.uint64(0xFFFF)).astype(np.uint16)
    return src.astype(np.uint32), dst.astype(np.uint32), sport, dp.astype(np.uint16), proto
