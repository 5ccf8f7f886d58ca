"""zipkin_amd — MI355X-native engine for Zipkin's dependency-link hot path."""
from .model import DependencyLink, Endpoint, Kind, Span, span2  # noqa: F401
