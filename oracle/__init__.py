"""ORACLE -- test infrastructure only (CPU restatement of the reference's path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/; the product package never does.
"""
