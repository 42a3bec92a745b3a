"""gRPC contract + transport helpers."""
from .schema import SERVICES, message, pb, service  # noqa: F401
from .server import RpcServer, serve_forever  # noqa: F401
from .client import Stub, channel  # noqa: F401
