"""Process groups, schedules and multi-rank runners."""

from .schedule import Phase, make_schedule, round_robin_rounds  # noqa: F401
from .session import create_session, dist_env, init_control_plane  # noqa: F401
