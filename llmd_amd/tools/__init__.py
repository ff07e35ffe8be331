"""Operator tools: calibration, flow-control tuning wizard, smoke healthcheck,
benchmark load generator."""
