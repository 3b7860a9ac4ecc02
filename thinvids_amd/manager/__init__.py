"""Manager: HTTP API + UI (:mod:`.app`), scheduler/watchdog/node logic (:mod:`.core`)."""
