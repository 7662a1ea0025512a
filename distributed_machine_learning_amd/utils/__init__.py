"""utils subsystem."""
