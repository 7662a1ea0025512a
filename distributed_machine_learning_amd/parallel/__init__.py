"""parallel subsystem."""
