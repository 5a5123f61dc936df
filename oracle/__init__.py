"""oracle — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package, and only as the checker (or the timed CPU baseline) — never as
the code path being measured or shipped.  The product (mdemi) never imports
it and has no CPU fallback.

Each function restates the reference's algorithm (pitlover/Monocular-Depth-
Estimation, mounted read-only at /root/reference in the build container) in
plain PyTorch CPU ops, NCHW like the reference, and cites the file:line it
follows.  Parity is pinned by tests/golden/*.npz, generated from the reference
itself by tests/golden/make_golden.py (tests/test_oracle_golden.py checks the
restatement against them).  Pieces the reference does not contain are marked
"parity unpinned": the EfficientNet-B5 encoder (torch.hub download, absent),
the SILog loss / optimizer / scheduler / train loop (run.py is missing).
"""
