"""ORACLE package — test infrastructure only (see ppo_oracle.py header).
Only tests/, __graft_entry__.smoke() and bench.py cpu_baseline may import it."""
