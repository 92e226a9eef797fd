"""ctypes binding of oracle/oracle.c (TEST INFRASTRUCTURE ONLY; see oracle/__init__.py)."""
import ctypes as C
import os

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "liboracle.so")


class ora_rule(C.Structure):
    _fields_ = [("action", C.c_int32), ("has_macip", C.c_uint8), ("has_ip_rule", C.c_uint8),
                ("has_ip", C.c_uint8), ("has_icmp", C.c_uint8), ("src", C.c_char_p), ("dst", C.c_char_p),
                ("tcp_present", C.c_uint8), ("tcp_has_src", C.c_uint8), ("tcp_has_dst", C.c_uint8),
                ("udp_present", C.c_uint8), ("udp_has_src", C.c_uint8), ("udp_has_dst", C.c_uint8),
                ("pad0", C.c_uint8), ("pad1", C.c_uint8),
                ("tcp_src_lo", C.c_uint32), ("tcp_src_hi", C.c_uint32), ("tcp_dst_lo", C.c_uint32),
                ("tcp_dst_hi", C.c_uint32), ("udp_src_lo", C.c_uint32), ("udp_src_hi", C.c_uint32),
                ("udp_dst_lo", C.c_uint32), ("udp_dst_hi", C.c_uint32)]


def _load():
    if not os.path.exists(_LIB):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(_LIB) + "/.."])
    lib = C.CDLL(_LIB)
    P = C.c_void_p
    lib.ora_eval_faithful.argtypes = [C.POINTER(ora_rule), C.c_int, P, P, P, P, C.c_size_t, P, P, C.c_int]
    lib.ora_acl_new.restype = P
    lib.ora_acl_new.argtypes = [C.POINTER(ora_rule), C.c_int]
    lib.ora_acl_free.argtypes = [P]
    lib.ora_eval.argtypes = [P, P, P, P, P, C.c_size_t, P, P, C.c_int]
    lib.ora_conn.argtypes = [P, P, P, P, P, P, P, P, P, P, C.c_size_t, P, P, P, P, P, C.c_int]
    lib.ora_perpod.argtypes = [P, P, P, P, P, P, P, C.c_size_t, P, P, P, C.c_int]
    lib.ora_conn_faithful.argtypes = [P, P, P, P, P, P, P, P, P, P, C.c_size_t, P, P, P, C.c_int]
    lib.ora_perpod_faithful.argtypes = [P, P, P, P, P, P, P, C.c_size_t, P, P, P, C.c_int]
    return lib


lib = _load()


def rules_from_dicts(rules):
    """ACL rule dicts ({"action","src","dst","tcp","udp",...}, as returned by
    vpp_amd Engine.GetACLByName or built by tests) -> ora_rule array (+ keepalive)."""
    arr = (ora_rule * max(1, len(rules)))()
    keep = []
    for i, r in enumerate(rules):
        x = arr[i]
        x.action = r["action"]
        x.has_macip = int(r.get("macip", False))
        x.has_ip_rule = int(r.get("ip_rule", True))
        x.has_ip = int(r.get("ip", True))
        x.has_icmp = int(r.get("icmp", False))
        s, d = (r.get("src") or "").encode(), (r.get("dst") or "").encode()
        keep += [s, d]
        x.src, x.dst = s, d
        for name in ("tcp", "udp"):
            sec = r.get(name)
            if sec:
                setattr(x, name + "_present", 1)
                if sec.get("src") is not None:
                    setattr(x, name + "_has_src", 1)
                    setattr(x, name + "_src_lo", sec["src"][0])
                    setattr(x, name + "_src_hi", sec["src"][1])
                if sec.get("dst") is not None:
                    setattr(x, name + "_has_dst", 1)
                    setattr(x, name + "_dst_lo", sec["dst"][0])
                    setattr(x, name + "_dst_hi", sec["dst"][1])
    return arr, keep


class ora_facl(C.Structure):
    _fields_ = [("r", C.POINTER(ora_rule)), ("n", C.c_int32)]


def _facls(acls):
    """the raw (string) rules of every table, for the faithful variants"""
    return (ora_facl * max(1, len(acls)))(*[ora_facl(a.arr, a.n) for a in acls])


class OraACL:
    def __init__(self, rules):
        self.arr, self.keep = rules_from_dicts(rules)
        self.n = len(rules)
        self.h = lib.ora_acl_new(self.arr, self.n)

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:  # lib is None at interpreter shutdown
            lib.ora_acl_free(self.h)
            self.h = None


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def eval_acl(acl, src, dst, dport, proto, threads=os.cpu_count() or 1):
    """evalACL over arrays -> (action int32[n], matched index int32[n] (-1 = none))."""
    n = len(src)
    src, dst = np.ascontiguousarray(src, np.uint32), np.ascontiguousarray(dst, np.uint32)
    dport, proto = np.ascontiguousarray(dport, np.uint16), np.ascontiguousarray(proto, np.uint8)
    act, idx = np.empty(n, np.int32), np.empty(n, np.int32)
    lib.ora_eval(acl.h if acl is not None else None, _p(src), _p(dst), _p(dport), _p(proto), n, _p(act), _p(idx),
                 threads)
    return act, idx


def eval_acl_faithful(rules_dicts, src, dst, dport, proto, threads=1):
    """evalACL with the rules' CIDR strings parsed on every rule visit (aclengine_mock.go:535, 549),
    one engine per thread over a slice of the tuples"""
    arr, keep = rules_from_dicts(rules_dicts)
    n = len(src)
    src, dst = np.ascontiguousarray(src, np.uint32), np.ascontiguousarray(dst, np.uint32)
    dport, proto = np.ascontiguousarray(dport, np.uint16), np.ascontiguousarray(proto, np.uint8)
    act, idx = np.empty(n, np.int32), np.empty(n, np.int32)
    lib.ora_eval_faithful(arr, len(rules_dicts), _p(src), _p(dst), _p(dport), _p(proto), n, _p(act), _p(idx),
                          threads)
    return act, idx


def test_connection(acls, if_in, if_out, sif, dif, src, dst, sport, dport, proto, threads=os.cpu_count() or 1,
                    trace=False, faithful=False):
    """testConnection per tuple over resolved interfaces. acls: list of OraACL (table id order).
    Returns (ConnAction, last evaluated table (-1 none/-2 unresolved), last matched index);
    trace=True also returns every evaluation the connection made, in the order
    aclengine_mock.go:448-491 makes them: (tables int32[n, 4], indices int32[n, 4]), table -3 =
    no evaluation, -2 = the unresolved-interface FAILURE, -1 = no ACL (nil: PERMIT).
    faithful=True: every evalACL parses its rules' CIDR strings on each rule visit, as
    aclengine_mock.go:535, 549 do (no trace; `threads` engines over slices of the tuples)."""
    n = len(src)
    harr = (C.c_void_p * max(1, len(acls)))(*[a.h for a in acls])
    cv = lambda a, dt: np.ascontiguousarray(a, dt)
    if_in, if_out, sif, dif = cv(if_in, np.int32), cv(if_out, np.int32), cv(sif, np.int32), cv(dif, np.int32)
    src, dst, sport, dport, proto = (cv(src, np.uint32), cv(dst, np.uint32), cv(sport, np.uint16),
                                     cv(dport, np.uint16), cv(proto, np.uint8))
    conn, lt, li = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32)
    if faithful:
        fa = _facls(acls)
        lib.ora_conn_faithful(C.cast(fa, C.c_void_p), _p(if_in), _p(if_out), _p(sif), _p(dif), _p(src), _p(dst),
                              _p(sport), _p(dport), _p(proto), n, _p(conn), _p(lt), _p(li), threads)
        return conn, lt, li
    evt = evi = None
    if trace:
        evt, evi = np.empty((n, 4), np.int32), np.empty((n, 4), np.int32)
    lib.ora_conn(C.cast(harr, C.c_void_p), _p(if_in), _p(if_out), _p(sif), _p(dif), _p(src), _p(dst), _p(sport),
                 _p(dport), _p(proto), n, _p(conn), _p(lt), _p(li), _p(evt) if trace else None,
                 _p(evi) if trace else None, threads)
    if trace:
        return conn, lt, li, evt, evi
    return conn, lt, li


def perpod(acls, if_out, dif, src, dst, dport, proto, threads=os.cpu_count() or 1, faithful=False):
    """evalACL(outbound ACL of the dst interface) per tuple. Returns (ACLAction, table
    (-1 = no ACL, -2 = unresolved interface), matched index (-1 = none)). faithful=True: CIDR
    strings parsed on each rule visit (aclengine_mock.go:535, 549)."""
    n = len(src)
    harr = (C.c_void_p * max(1, len(acls)))(*[a.h for a in acls])
    cv = lambda a, dt: np.ascontiguousarray(a, dt)
    if_out, dif = cv(if_out, np.int32), cv(dif, np.int32)
    src, dst, dport, proto = cv(src, np.uint32), cv(dst, np.uint32), cv(dport, np.uint16), cv(proto, np.uint8)
    act, lt, li = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32)
    if faithful:
        fa = _facls(acls)
        lib.ora_perpod_faithful(C.cast(fa, C.c_void_p), _p(if_out), _p(dif), _p(src), _p(dst), _p(dport), _p(proto),
                                n, _p(act), _p(lt), _p(li), threads)
        return act, lt, li
    lib.ora_perpod(C.cast(harr, C.c_void_p), _p(if_out), _p(dif), _p(src), _p(dst), _p(dport), _p(proto), n,
                   _p(act), _p(lt), _p(li), threads)
    return act, lt, li
