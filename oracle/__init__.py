"""ORACLE — TEST INFRASTRUCTURE ONLY.

This package is the CPU restatement of the reference VAESNe training step
(YunyiShen/VAESNe-dev, `package/VAESNe/*.py`).  It exists so that `tests/`,
`__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` have an
independent checker.  The product path (`vaesne-dev_amd/VAESNe`) never imports
it and has no CPU fallback.

Pinning: `tests/golden/*.npz` are produced by `tests/golden/gen_golden.py`,
which imports the *reference* package in a separate process.  `tests/
test_oracle_golden.py` checks this restatement against those fixtures.
"""
