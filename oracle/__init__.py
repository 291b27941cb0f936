"""TEST INFRASTRUCTURE ONLY — CPU oracle of the single-node flip walk.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package.  The product package ``flipcomplexityempirical_amd``
never imports it; its HIP path fails loudly when the extension is missing.

* ``oracle.oracle``          ctypes wrapper of ``flipchain_oracle.c`` (C restatement,
                             trajectory-exact with the HIP path)
* ``oracle.reference_proxy`` pure-Python GerryChain-equivalent proxy (dict copy per
                             proposal, cut-edge sets, networkx Dijkstra contiguity):
                             the "reference CPU path" timed beside the GPU
"""
