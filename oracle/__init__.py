"""CPU oracle — TEST INFRASTRUCTURE ONLY (see numpy_ref.py). Never imported by fedn_amd."""
