"""Native (HIP / gfx950) operator wrappers."""
