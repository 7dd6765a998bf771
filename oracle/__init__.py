"""CPU oracle -- TEST INFRASTRUCTURE ONLY (see oracle/oracle.py and fc_oracle.c headers).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
