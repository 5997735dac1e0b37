"""Test-infrastructure oracle (CPU restatement of the reference hot path). See nerf_oracle.py header."""
