"""CPU oracle for the network-policy classification path -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU and independently of the product code in
``vpp_amd/``, the reference algorithm of Contiv-VPP's policy path:

* ``gonet``      -- Go 1.11 ``net`` semantics used by the path (ParseCIDR, Contains,
                    IPNet.String) -- SURVEY.md §8a row a15.
* ``policy``     -- ContivRule ordering, ContivRuleTable, the renderer cache in both
                    orientations, and the ACL renderer (rows a1-a8).
* ``aclengine``  -- the mock ACL engine: ApplyTxn/PutACL/DelACL, evalACL with the
                    matched rule index, testConnection and Connection* (rows a10-a12).
* ``mockrenderer`` -- mock/renderer TestTraffic (row a13).
* ``configurator`` -- the policy configurator + mock renderer (row f1).
* ``k8s_policy`` -- the K8s policy cache (label / namespace selector expansion) and the
                    policy processor (row f3).
* ``fast``       -- ctypes binding of ``oracle/oracle.c``: the same evalACL /
                    testConnection restated in C for bulk parity checks and the CPU
                    baseline leg of bench.py.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker -- never as the thing measured or shipped.

Pinning: the restatement is checked against the reference's own known-answer tests,
transcribed as data into ``tests/golden/`` by ``tests/golden/make_golden.py``
(acl_renderer_test.go Connection* verdicts, ACL counts/placement, and
cache_test.go ordered rule tables).
"""
