"""CPU oracle — TEST INFRASTRUCTURE ONLY (see ref_kf.py). Never imported by the product path."""
