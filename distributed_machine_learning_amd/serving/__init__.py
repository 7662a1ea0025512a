"""serving subsystem."""
