"""TEST INFRASTRUCTURE: CPU oracle of the IMPALA learner step (see oracle/oracle.py)."""
