"""The measured parity figures of the -m gpu suite (DESIGN.md §3 cites them): every GPU test may
add an entry; tests/conftest.py writes the dict to gpurun_out/parity_report.json when the session
ends (if any test added one)."""
REPORT = {}
