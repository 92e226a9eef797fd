"""The reference's acl_renderer_test.go, replayed through the product on the GPU: the C++
renderer renders the transactions, the device engine installs the ACLs, and all 284
Connection* verdicts are evaluated by the testConnection kernel (plus every ACL count /
change count / reflective + global ACL placement assertion)."""
import pytest

import kat_driver as kd

pytestmark = pytest.mark.gpu

SCENARIOS = kd.load("acl_renderer_kats.json")


@pytest.mark.parametrize("sc", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_acl_renderer_kats_on_gpu(sc):
    seen = []
    bad = kd.run_scenario(kd.ProductBackend(gpu=True), sc, on_check=lambda c, g, ok: seen.append(c["kind"]))
    assert not bad, bad[:5]
    assert sum(1 for k in seen if k.startswith("Connection")) == sum(
        1 for p in sc["phases"] for c in p["checks"] if c["kind"].startswith("Connection"))
