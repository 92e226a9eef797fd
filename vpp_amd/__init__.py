"""vpp_amd -- MI355X-native network-policy classification engine for Contiv-VPP's policy path.

Layout:
  csrc/        C++17 host side (renderer cache, ACL renderer, engine, compiler) + gfx950 HIP
               kernels, built into libpolicygpu.so behind the C ABI of include/policygpu.h
  _capi.py     ctypes binding of that ABI (no fallback: missing library = ImportError)
  renderer.py  the reference-shaped Python face (PolicyRendererAPI, MockACLEngine API)
  workloads.py synthetic workloads of BASELINE.json configs 1-5
  device.py    device-buffer helpers (torch used only for HBM allocation and streams)
"""
from . import _capi  # noqa: F401  (loads libpolicygpu.so or raises)
from .renderer import (ANY, OTHER, TCP, UDP, ActionDeny, ActionPermit, ConnActionAllow,  # noqa: F401
                       ConnActionDenySyn, ConnActionDenySynAck, ConnActionFailure, ContivRule, Engine,
                       EgressOrientation, IngressOrientation, IPNet, PolicyError, Renderer)
