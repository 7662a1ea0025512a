"""cluster subsystem."""
