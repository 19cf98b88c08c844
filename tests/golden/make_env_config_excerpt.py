"""Extract the constants the reference dumped for one of its training runs (data, not code)
into tests/golden/env_config_excerpt.json.  Run in the container that mounts /root/reference."""
import json
import os
import re

SRC = ("/root/reference/train_results_phoenix/DroneHoverBulletFreeEnvWithoutAdversary-v0/ppo/"
       "2023_11_24_10_46/seed_61305/env_config.json")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "env_config_excerpt.json")


def find(d, key):
    if isinstance(d, dict):
        for k, v in d.items():
            if k == key:
                return v
            r = find(v, key)
            if r is not None:
                return r
    return None


def main():
    d = json.load(open(SRC))
    # the dump nests the agent under input_parameters.self.<env repr>.drone.<agent repr>
    env = next(iter(d["input_parameters"]["self"].values()))
    drone = next(iter(env["drone"].values()))
    def arr(s):
        return [float(x) for x in re.findall(r"[-+0-9.e]+", s)] if isinstance(s, str) else s
    out = {
        "source": SRC.replace("/root/reference/", ""),
        "K": drone["K"], "A": arr(drone["A"])[0], "B": arr(drone["B"])[0],
        "HOVER_X": drone["HOVER_X"], "HOVER_ACTION": drone["HOVER_ACTION"], "buf_size": drone["buf_size"],
        "J_diag": [drone["IXX"], drone["IYY"], drone["IZZ"]], "M": drone["M"],
        "DRAG_COEFF": arr(drone["DRAG_COEFF"]), "TIME_STEP": d["TIME_STEP"],
        "domain_randomization": d["domain_randomization"],
        "motor_thrust_noise": d["agent_params"]["motor_thrust_noise"],
        "MAX_THRUST": drone["MAX_THRUST"], "GRAVITY": drone["GRAVITY"],
    }
    json.dump(out, open(OUT, "w"), indent=1)
    print(out)


if __name__ == "__main__":
    main()
