"""OpenAI-compatible server with vLLM's command line (``api_server``)."""
