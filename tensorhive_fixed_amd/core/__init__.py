"""Daemon runtime: transports, telemetry, services, scheduling, task supervision."""
