"""Constructor keyword arguments of the reference env -> SngConfig.

Same names, defaults and parsing as SmartNanogridEnv.__init__ / set_time_interval
(smart_nanogrid_environment.py:32-138); the reference's hard-coded module constants
(BESS, EV, tariffs, penalty weights) become overridable fields with the reference values.
"""
import ctypes

from . import _native

PENALTY_MODES = {"no_penalty": 0, "on_departure": 1, "sparse": 2, "dense": 3}

WRONG_PENALTY_MODE = "Error: Wrong vehicle uncharged - penalty mode provided!"   # charging_station.py:60
WRONG_CHARGING_MODE = "Error: Wrong charging mode provided!"                     # charger.py:88
NEGATIVE_DEMAND = "Error: If V2X mode is not enabled, then power_demand cannot be less than 0!"  # central_management_system.py:159
BESS_ABOVE_ONE = "Error: Battery SOC greater than 1!"                              # penaliser.py:111


def parse_time_interval(requested_time_interval):
    """set_time_interval (smart_nanogrid_environment.py:125-138): '1h' -> 1.0, '15min' -> 0.25, '' -> 1.0."""
    if requested_time_interval:
        if "h" in requested_time_interval:
            return float(requested_time_interval.replace("h", ""))
        if "min" in requested_time_interval:
            return float(requested_time_interval.replace("min", "")) / 60.0
        raise ValueError("Wrong time interval was provided")
    return float(1)


class EnvSettings:
    def __init__(self, price_model=0, number_of_chargers=8, pv_system_available_in_model=True,
                 battery_system_available_in_model=True, vehicle_to_everything=False,
                 enable_different_vehicle_battery_capacities=True, enable_requested_state_of_charge=False,
                 algorithm_used="", environment_mode="", time_interval="", charging_mode="",
                 vehicle_uncharged_penalty_mode="", numpy_legacy_promotion=False, grid_cost_weight=0.75,
                 **constants):
        if price_model == 5:   # accountant.py:90-98 indexes a list with a tuple
            raise TypeError("list indices must be integers or slices, not tuple")
        if price_model not in (0, 1, 2, 3, 4):
            raise ValueError(f"unsupported price_model {price_model!r}")
        self.price_model = int(price_model)
        self.number_of_chargers = int(number_of_chargers)
        self.pv = bool(pv_system_available_in_model)
        self.bess = bool(battery_system_available_in_model)
        self.v2x = bool(vehicle_to_everything)
        self.different_capacities = bool(enable_different_vehicle_battery_capacities)
        self.requested_soc = bool(enable_requested_state_of_charge)
        self.algorithm_used = algorithm_used
        self.environment_mode = environment_mode
        self.requested_time_interval = time_interval
        self.time_interval = parse_time_interval(time_interval)
        self.charging_mode = charging_mode
        self.penalty_mode_name = vehicle_uncharged_penalty_mode
        self.penalty_mode = PENALTY_MODES.get(vehicle_uncharged_penalty_mode)   # None: raises at reset
        self.numpy_legacy_promotion = bool(numpy_legacy_promotion)
        self.grid_cost_weight = float(grid_cost_weight)
        self.constants = constants
        self.timesteps = int(24 / self.time_interval)
        self.obs_dim = (1 + int(self.pv)) * 4 + 2 * self.number_of_chargers + int(self.bess)
        self.act_dim = self.number_of_chargers + int(self.bess)

    def to_native(self):
        L = _native.lib()
        cfg = _native.SngConfig()
        L.sng_config_defaults(ctypes.byref(cfg))
        cfg.number_of_chargers = self.number_of_chargers
        cfg.time_interval_hours = self.time_interval
        cfg.price_model = self.price_model
        cfg.pv_system_available = int(self.pv)
        cfg.battery_system_available = int(self.bess)
        cfg.vehicle_to_everything = int(self.v2x)
        cfg.different_vehicle_capacities = int(self.different_capacities)
        cfg.requested_state_of_charge = int(self.requested_soc)
        cfg.charging_mode_bounded = int(self.charging_mode == "bounded")
        cfg.penalty_mode = self.penalty_mode if self.penalty_mode is not None else 0
        cfg.numpy_legacy_promotion = int(self.numpy_legacy_promotion)
        cfg.grid_cost_weight = self.grid_cost_weight
        for k, v in self.constants.items():
            if not hasattr(cfg, k):
                raise TypeError(f"unexpected keyword argument {k!r}")
            setattr(cfg, k, v)
        irr = _native.load_irradiance()
        self._irr = irr   # keep alive for the duration of sng_create
        cfg.irradiance_per_minute = irr.ctypes.data_as(_native.c_double_p)
        cfg.irradiance_minutes = irr.size
        return cfg

    def variant_name(self):
        """smart_nanogrid_environment.py:280-287"""
        if self.bess and self.pv and self.v2x:
            return "v2x-b-pv"
        if self.v2x:
            return "v2x"
        if self.bess and self.pv:
            return "b-pv"
        return "basic"
