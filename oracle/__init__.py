"""CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import anything from this package.  The product package ``dcvc_amd`` must
never import it (tests/test_boundary.py checks this).
"""
