"""ORACLE — test infrastructure only (see dl_oracle.py header). Not imported by zipkin_amd."""
