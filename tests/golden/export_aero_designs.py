"""Export the reference's test designs WITH their rotor tables (blade, airfoils, control and
operating schedule) as JSON fixtures, for the wind cases of the reference's
tests/test_model.py (desired_X0 'wind' / 'wind_wave_current', desired_fn 'loaded').

Only the YAML inputs are read (yaml.SafeLoader); nothing of the reference is imported.  The
GPU box has no /root/reference, so the fixtures are committed under tests/golden/designs/.

    python tests/golden/export_aero_designs.py
"""
import json
import os

import yaml

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
DESIGNS = {
    "VolturnUS-S_aero": "tests/test_data/VolturnUS-S.yaml",
    "OC3spar_aero": "tests/test_data/OC3spar.yaml",
    "VolturnUS-S_farm_aero": "tests/test_data/VolturnUS-S_farm.yaml",
}


def main():
    for name, rel in DESIGNS.items():
        with open(os.path.join(REF, rel)) as f:
            d = yaml.load(f, Loader=yaml.SafeLoader)
        if "array_mooring" in d:     # the MoorDyn-style file is already a fixture (designs/)
            d["array_mooring"] = {"file": os.path.basename(d["array_mooring"]["file"])}
        with open(os.path.join(HERE, "designs", name + ".json"), "w") as f:
            json.dump(d, f, indent=1, default=str)
        print("wrote", name)


if __name__ == "__main__":
    main()
