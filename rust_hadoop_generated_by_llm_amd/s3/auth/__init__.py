"""S3 authentication & authorisation (reference dfs/common/src/auth/)."""
from .errors import AuthError  # noqa: F401
