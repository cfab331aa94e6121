"""Oracle package -- TEST INFRASTRUCTURE ONLY (see filters_oracle.py)."""
