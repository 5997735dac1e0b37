def FormatCode(text, style_config=None, **kwargs):
    """No-op formatter stand-in (golden generator only)."""
    return text, False
