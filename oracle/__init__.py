"""Test oracle (CPU restatements). Importable only from tests/, smoke() and bench.py's cpu_baseline."""
