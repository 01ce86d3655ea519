"""REST API: spec-driven router/validator, JWT auth, response catalogue."""
