"""Import-only stand-in (the reference's plotting imports networkx; nothing here draws)."""
