"""CPU oracle — TEST INFRASTRUCTURE ONLY (see ``cfsd_oracle.py`` header)."""
