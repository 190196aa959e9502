"""Host-side utilities (dedispersion planning)."""
