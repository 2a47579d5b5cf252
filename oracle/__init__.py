"""ORACLE — test infrastructure only.

CPU restatements of the reference algorithms this repo accelerates, used solely as the
checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing under
tts-3_amd/ imports this package; the product path has no CPU fallback.
"""
