"""HBM tuple batches and kernel launches.

torch is used only as the allocator of device memory and for streams/events (HIP under
ROCm); the compute is the C-ABI kernels. Tuples are SoA:
  src_ip u32, dst_ip u32, dport u16, proto u8 (+ sport u16 for connection mode).
"""
import ctypes as C

import numpy as np
import torch

from . import _capi
from ._capi import lib


class TupleBatch:
    def __init__(self, n, device="cuda", with_sport=True):
        self.n = n
        self.src = torch.empty(n, dtype=torch.int32, device=device)
        self.dst = torch.empty(n, dtype=torch.int32, device=device)
        self.dport = torch.empty(n, dtype=torch.int16, device=device)
        self.proto = torch.empty(n, dtype=torch.uint8, device=device)
        self.sport = torch.empty(n, dtype=torch.int16, device=device) if with_sport else None

    @classmethod
    def from_numpy(cls, src, dst, sport, dport, proto, device="cuda"):
        b = cls.__new__(cls)
        b.n = len(src)
        b.src = torch.from_numpy(np.ascontiguousarray(src, dtype=np.uint32).view(np.int32)).to(device)
        b.dst = torch.from_numpy(np.ascontiguousarray(dst, dtype=np.uint32).view(np.int32)).to(device)
        b.dport = torch.from_numpy(np.ascontiguousarray(dport, dtype=np.uint16).view(np.int16)).to(device)
        b.proto = torch.from_numpy(np.ascontiguousarray(proto, dtype=np.uint8)).to(device)
        b.sport = torch.from_numpy(np.ascontiguousarray(sport, dtype=np.uint16).view(np.int16)).to(device)
        return b

    def soa(self, offset=0):
        s = _capi.pg_tuple_soa()
        s.src_ip = self.src.data_ptr() + 4 * offset
        s.dst_ip = self.dst.data_ptr() + 4 * offset
        s.dst_port = self.dport.data_ptr() + 2 * offset
        s.proto = self.proto.data_ptr() + offset
        s.src_port = (self.sport.data_ptr() + 2 * offset) if self.sport is not None else None
        return s

    def numpy(self, k=None):
        k = self.n if k is None else k
        g = lambda t, dt: t[:k].cpu().numpy().view(dt)
        return (g(self.src, np.uint32), g(self.dst, np.uint32),
                g(self.sport, np.uint16) if self.sport is not None else np.zeros(k, np.uint16),
                g(self.dport, np.uint16), g(self.proto, np.uint8))


def _stream_ptr(stream):
    if stream is None:
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    return C.c_void_p(stream.cuda_stream)


def gen_tuples(engine, batch, seed, table_id=-1, inside_pct=0, ip_pool=None, pool_pct=0, dst_pool_pct=0,
               port_pool=None, port_pool_pct=0, tcp_pct=45, udp_pct=45, zipf_cdf=None, nomatch_pct=0,
               index_base=0, stream=None):
    spec = _capi.pg_gen_spec()
    spec.seed, spec.index_base, spec.table_id, spec.inside_pct = seed, index_base, table_id, inside_pct
    keep = []
    if ip_pool is not None and len(ip_pool):
        a = np.ascontiguousarray(ip_pool, dtype=np.uint32)
        keep.append(a)
        spec.ip_pool = a.ctypes.data_as(C.POINTER(C.c_uint32))
        spec.n_ip_pool = len(a)
    if port_pool is not None and len(port_pool):
        p = np.ascontiguousarray(port_pool, dtype=np.uint16)
        keep.append(p)
        spec.port_pool = p.ctypes.data_as(C.POINTER(C.c_uint16))
        spec.n_port_pool = len(p)
    if zipf_cdf is not None:
        z = np.ascontiguousarray(zipf_cdf, dtype=np.uint32)
        keep.append(z)
        spec.zipf_cdf = z.ctypes.data_as(C.POINTER(C.c_uint32))
    spec.pool_pct, spec.dst_pool_pct, spec.port_pool_pct = pool_pct, dst_pool_pct, port_pool_pct
    spec.tcp_pct, spec.udp_pct, spec.nomatch_pct = tcp_pct, udp_pct, nomatch_pct
    sp = batch.sport.data_ptr() if batch.sport is not None else None
    engine._ck(lib.pg_gen_tuples(engine.h, C.byref(spec), batch.n, batch.src.data_ptr(), batch.dst.data_ptr(),
                                 sp, batch.dport.data_ptr(), batch.proto.data_ptr(), _stream_ptr(stream)))


def classify(engine, mode, table_id, batch, out, counters=None, stream=None, offset=0, n=None):
    n = batch.n - offset if n is None else n
    soa = batch.soa(offset)
    cptr = counters if (counters is None or isinstance(counters, int)) else counters.data_ptr()
    engine._ck(lib.pg_classify(engine.h, mode, table_id, C.byref(soa), n, out.data_ptr() + 4 * offset, cptr,
                               _stream_ptr(stream)))


def classify_linear(engine, table_id, batch, out, stream=None):
    soa = batch.soa()
    engine._ck(lib.pg_classify_linear(engine.h, table_id, C.byref(soa), batch.n, out.data_ptr(),
                                      _stream_ptr(stream)))


def stream_probe(engine, fields, batch, out, stream=None):
    """pg_stream_probe: the loads and store of a classify launch over `batch` without the
    classification (fields: 1 = dst, 2 = sport) -- a measurement, not a classification"""
    soa = batch.soa()
    engine._ck(lib.pg_stream_probe(engine.h, fields, C.byref(soa), batch.n, out.data_ptr(), _stream_ptr(stream)))


def counters_device_ptr(engine):
    p = lib.pg_counters_device(engine.h)
    if not p:
        raise RuntimeError(lib.pg_last_error(engine.h).decode())
    return p


def read_counters(engine):
    n = engine.num_counter_slots()
    buf = (C.c_uint64 * n)()
    engine._ck(lib.pg_read_counters(engine.h, buf, n))
    return np.frombuffer(buf, dtype=np.uint64).copy()


def reset_counters(engine, stream=None):
    engine._ck(lib.pg_reset_counters(engine.h, _stream_ptr(stream)))


def counters_snapshot(engine):
    """the gauge snapshot (pg_counters_snapshot: the cluster sum once a communicator exists,
    else this GPU's counts as of the last read; no GPU access)"""
    n = engine._ck(lib.pg_counters_snapshot(engine.h, None, 0))
    buf = (C.c_uint64 * max(1, n))()
    engine._ck(lib.pg_counters_snapshot(engine.h, buf, n))
    return np.frombuffer(buf, dtype=np.uint64)[:n].copy()


def counters_snapshot_range(engine, which, first, n):
    """slots [first, first + n) of a host snapshot (SNAP_LOCAL / SNAP_CLUSTER / SNAP_GAUGE)
    -> (u64 array, its layout generation); no GPU access"""
    buf = (C.c_uint64 * max(1, n))()
    gen = C.c_uint64()
    k = engine._ck(lib.pg_counters_snapshot_range(engine.h, which, first, n, buf, C.byref(gen)))
    return np.frombuffer(buf, dtype=np.uint64)[:k].copy(), gen.value


def counter_of_rule(engine, which, acl_name, rule_index):
    """one rule's count in a host snapshot by (ACL name, rule index; -1 = default deny; name
    None: -1 "no ACL", -2 unresolved) resolved in that snapshot's layout -> (value, layout
    generation), or None when the snapshot has no such rule; no GPU access"""
    v, gen = C.c_uint64(), C.c_uint64()
    rc = lib.pg_counter_of_rule(engine.h, which, acl_name.encode() if acl_name is not None else None, rule_index,
                                C.byref(v), C.byref(gen))
    if rc == _capi.PG_ENOENT:
        return None
    engine._ck(rc)
    return v.value, gen.value


def counter_layout_gen(engine):
    return lib.pg_counter_layout_gen(engine.h)


# ---- RCCL counter all-reduce through the C ABI (include/policygpu.h pg_comm_*) -------------
def comm_unique_id():
    buf = C.create_string_buffer(128)
    rc = lib.pg_comm_unique_id(buf)
    if rc < 0:
        raise RuntimeError("pg_comm_unique_id failed (%d)" % rc)
    return buf.raw


def comm_init_rank(engine, nranks, uid, rank):
    engine._ck(lib.pg_comm_init_rank(engine.h, nranks, C.create_string_buffer(uid, 128), rank))


def comm_init_all(engines):
    arr = (C.c_void_p * len(engines))(*[e.h for e in engines])
    rc = lib.pg_comm_init_all(arr, len(engines))
    if rc < 0:
        engines[0]._ck(rc)


def allreduce_counters(engine, stream=None):
    """sum this rank's device counters over the communicator -> the summed counters (the
    device counters themselves keep this rank's counts)"""
    engine._ck(lib.pg_allreduce_counters(engine.h, _stream_ptr(stream)))
    return counters_snapshot(engine)


def allreduce_counters_all(engines):
    arr = (C.c_void_p * len(engines))(*[e.h for e in engines])
    rc = lib.pg_allreduce_counters_all(arr, len(engines))
    if rc < 0:
        for e in engines:
            msg = lib.pg_last_error(e.h).decode()
            if msg:
                raise RuntimeError("%s (code %d)" % (msg, rc))
        raise RuntimeError("pg_allreduce_counters_all failed (%d)" % rc)
    return [counters_snapshot(e) for e in engines]


def unpack(out_u32):
    w = out_u32.astype(np.uint32)
    return (w >> 30).astype(np.int64), (w & 0x3FFFFFFF).astype(np.int64)
