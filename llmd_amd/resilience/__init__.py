"""Resilience: the Inference Resilience Operator (``operator.py``)."""
