"""Parity oracle (CPU restatement of the reference hot path) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package.  The product (moeva2-ijcai22-replication_amd/) never does.
"""
