"""§8 a13 on the device: MockRenderer.TestTraffic (mock/renderer/renderer_mock.go:105-147) of
the configurator's rendered lists, answered by k_classify (SINGLE mode) after
pg_mock_renderer_install, checked against

* the 174 TestTraffic assertions of configurator_test.go (tests/golden/configurator_kats.json),
* the host TestTraffic (itself pinned by those KATs) on random configurator scenarios.

The CPU tests run the kernels' per-tuple code on the host (pg_debug_classify_host), the GPU
tests k_classify."""
import random

import kat_driver as kd
import numpy as np
import pytest

from test_configurator import EXPECT, FIX, TRAFFIC, rand_scenario, run_product
from vpp_amd import configurator as CF
from vpp_amd import renderer as R
from vpp_amd import workloads as W


def _groups(traffic):
    g = {}
    for t in traffic:
        g.setdefault((t["renderer"], t["pod"], TRAFFIC[t["direction"]]), []).append(t)
    return g


def _device_traffic(e, mock, pod, direction, pk, classify):
    """TrafficAction of packets pk = (src u32, dst u32, proto, sport, dport) via the device path"""
    name = "traffic-%s-%d" % (pod.replace("/", "-"), direction)
    tid = mock.InstallTraffic(e, pod, direction, name)
    if tid is None:
        return np.full(len(pk[0]), 2)
    got = classify(e, tid, *pk)
    return CF.MockRenderer.TrafficOf(e, tid, got)


def _host_classify(e, tid, src, dst, proto, sport, dport):
    return e.debug_classify_host(0, tid, src, dst, sport, dport, proto)


def _gpu_classify(e, tid, src, dst, proto, sport, dport):
    import torch
    from vpp_amd import device as D
    n = len(src)
    b = D.TupleBatch.from_numpy(src, dst, sport, dport, proto)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    D.classify(e, 0, tid, b, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def _kats(classify):
    bad, n = [], 0
    for sc in FIX:
        _, mocks = run_product(sc)
        e = R.Engine(0)
        for (r, pod, direction), ts in _groups(sc["traffic"]).items():
            pk = (np.array([W.ip_u32(t["src"]) for t in ts], np.uint32),
                  np.array([W.ip_u32(t["dst"]) for t in ts], np.uint32),
                  np.array([kd.PROTO[t["proto"]] for t in ts], np.uint8),
                  np.array([t["sport"] for t in ts], np.uint16), np.array([t["dport"] for t in ts], np.uint16))
            got = _device_traffic(e, mocks[r], pod, direction, pk, classify)
            for t, g in zip(ts, got):
                n += 1
                if g != EXPECT[t["expect"]]:
                    bad.append("configurator_test.go:%d" % t["line"])
    return bad, n


def test_testtraffic_kats_host():
    bad, n = _kats(_host_classify)
    assert n == 174 and not bad, bad


def _random_case(seed, classify, n=2000):
    rnd = random.Random(4000 + seed)
    sc = rand_scenario(rnd)
    cfg = CF.PolicyConfigurator()
    for pod, ip in sc["pods"].items():
        if ip is not None:
            cfg.AddPodConfig(pod, ip)
    cfg.SetNatLoopbackIP(sc["nat"])
    mock = CF.MockRenderer()
    assert cfg.RegisterRenderer(mock) is None
    txn = cfg.NewTxn(sc["txn"]["resync"])
    from test_configurator import product_policy
    for pod, plist in sc["txn"]["configure"]:
        txn.Configure(pod, [product_policy(sc["policies"][v]) for v in plist])
    assert txn.Commit() is None
    e = R.Engine(0)
    rng = np.random.default_rng(seed)
    ips = [W.ip_u32(ip) for ip in sc["pods"].values() if ip] + [W.ip_u32("8.8.8.8"), W.ip_u32("10.0.0.1")]
    checked = 0
    for pod in sc["pods"]:
        for direction in (0, 1):
            src = np.where(rng.random(n) < 0.7, np.array(ips, np.uint32)[rng.integers(0, len(ips), n)],
                           rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))
            dst = np.where(rng.random(n) < 0.7, np.array(ips, np.uint32)[rng.integers(0, len(ips), n)],
                           rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))
            proto = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.5, 0.4, 0.1])
            sport = rng.integers(0, 1 << 16, n).astype(np.uint16)
            dport = np.where(rng.random(n) < 0.6, rng.choice(np.array([22, 53, 80, 443, 8080], np.uint16), n),
                             rng.integers(0, 1 << 16, n)).astype(np.uint16)
            got = _device_traffic(e, mock, pod, direction, (src, dst, proto, sport, dport), classify)
            want = [mock.TestTraffic(pod, direction, W.ip_str(int(s)), W.ip_str(int(d)), int(p), int(sp), int(dp))
                    for s, d, p, sp, dp in zip(src, dst, proto, sport, dport)]
            assert list(got) == want, (pod, direction)
            checked += 1
    return checked


@pytest.mark.parametrize("seed", range(5))
def test_testtraffic_random_host(seed):
    assert _random_case(seed, _host_classify, n=600) > 0


@pytest.mark.gpu
def test_testtraffic_kats_gpu():
    bad, n = _kats(_gpu_classify)
    assert n == 174 and not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_testtraffic_random_gpu(seed):
    assert _random_case(seed, _gpu_classify) > 0
