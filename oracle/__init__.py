"""CPU oracle for the capk hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain PyTorch-CPU, fp32 restatement of the reference's
image-captioning hot path (thromel/Image-Captioning-ML-Project, mounted
read-only at /root/reference in the build container; it never travels to the
GPU box).  Every function cites the reference file:line (or the pinned
third-party file it delegates to: torch 2.10.0 / transformers 5.15.0) whose
arithmetic it restates, including the minimal fixes for the reference defects
catalogued in SURVEY.md §0.1 (D1..D16).

Who may use it:  only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — and there only as the *checker* or as the
timed CPU baseline, never as the thing measured or shipped.  The product path
(``image-captioning-ml-project_amd/capk``) never imports this package.

Pinning: the restatement is checked against golden vectors produced by running
the reference code itself in the build container (``oracle/gen_golden.py`` ->
``tests/golden/*.npz``); see ``tests/test_oracle_golden.py``.
"""
