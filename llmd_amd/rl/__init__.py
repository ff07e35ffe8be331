"""RL integration: collaborative GPU time-slicing (``timeslice.py``); weight sync lives in engine/weight_sync.py."""
