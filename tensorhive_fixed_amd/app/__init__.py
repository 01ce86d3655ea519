"""Web dashboard server (static SPA + ``static/config.json``)."""
