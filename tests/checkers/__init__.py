"""Test-only checkers (torch restatements of third-party reference code)."""
