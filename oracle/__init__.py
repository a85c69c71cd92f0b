"""CPU restatement of the koord-scheduler Filter/Score path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
The product path (koordinator_amd) never loads it.  See koord_oracle.c for the reference
file:line each function restates.
"""
