"""store subsystem."""
