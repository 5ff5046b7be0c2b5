"""TEST INFRASTRUCTURE ONLY — CPU oracle for rankops parity.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package; the product (rankops) never does.

PARITY UNPINNED: the reference ships no tests, golden vectors or known-answer fixtures for
this path, and it may not be imported or run here (SURVEY.md §8c records the permission
denial).  `reference_forward` is therefore a line-by-line CPU restatement (plain PyTorch fp32,
the same ATen ops in the same order) of the cited reference lines; it is cross-checked only
against an independent float64 numpy restatement (`reference_np`) and against the committed
fixtures under tests/golden/, which it generated itself.
"""
