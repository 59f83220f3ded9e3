"""`solver` CLI: load device/model profiles, run halda_solve on the GPU, print/save.

Same surface and output as the reference CLI (src/cli/solver.py:15-237):
  * --profile <folder> (falls back to test/profiles/<folder> relative to the
    working directory), or --devices ... --model ...;
  * device files sorted by name, device 0 forced to is_head=True;
  * model JSON either ModelProfileSplit (f_q has prefill/decode) -> decode-phase
    ModelProfile, or a plain ModelProfile;
  * halda_solve(devices, model, mip_gap=args.mip_gap, plot=not args.no_plot,
    kv_bits="4bit") — kv_bits is fixed to "4bit" as in the reference (:211);
    --time-limit / --max-iters / --sdisk-threshold / --k-candidates are accepted
    and ignored, as in the reference;
  * --quiet / --verbose / --save-solution formats of :176-235.
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path
from typing import List, Tuple

from ..common import DeviceProfile, ModelProfile, ModelProfileSplit
from ..solver import halda_solve


def load_device_profile(device_path: str) -> DeviceProfile:
    return DeviceProfile.model_validate(json.loads(Path(device_path).read_text()))


def load_model_profile(model_path: str) -> ModelProfile:
    data = json.loads(Path(model_path).read_text())
    f_q = data.get("f_q")
    if isinstance(f_q, dict) and "prefill" in f_q and "decode" in f_q:
        return ModelProfileSplit.model_validate(data).to_model_profile()
    return ModelProfile.model_validate(data)


def load_devices_and_model(device_files: List[str], model_file: str) -> Tuple[List[DeviceProfile], ModelProfile]:
    devices = [load_device_profile(f) for f in device_files]
    if devices:
        devices[0].is_head = True
    return devices, load_model_profile(model_file)


def load_from_profile_folder(profile_path: str):
    folder = Path(profile_path)
    if not folder.exists():
        folder = Path("test/profiles") / profile_path
        if not folder.exists():
            raise FileNotFoundError(f"Profile folder not found: {profile_path}")
    model_file = folder / "model_profile.json"
    if not model_file.exists():
        raise FileNotFoundError(f"model_profile.json not found in {folder}")
    device_files = sorted(str(f) for f in folder.glob("*.json") if f.name != "model_profile.json")
    if not device_files:
        raise ValueError(f"No device profiles found in {folder}")
    return load_devices_and_model(device_files, str(model_file))


def _parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Run HALDA solver for distributed LLM inference optimization",
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    src = p.add_mutually_exclusive_group(required=True)
    src.add_argument("--devices", nargs="+", help="Device profile JSON files (requires --model)")
    src.add_argument("--profile", help="Profile folder path (e.g., 'hermes_70b' or 'profiles/hermes_70b')")
    p.add_argument("--model", help="Model profile JSON file (required with --devices)")
    g = p.add_argument_group("solver parameters")
    g.add_argument("--time-limit", type=float, default=5.0, help="Time limit per k value in seconds (default: 5.0)")
    g.add_argument("--max-iters", type=int, default=50, help="Maximum outer iterations (default: 50)")
    g.add_argument("--mip-gap", type=float, default=1e-4, help="MIP gap tolerance (default: 1e-4)")
    g.add_argument("--sdisk-threshold", type=float, help="Disk speed threshold for forcing devices to M4 (bytes/s)")
    g.add_argument("--k-candidates", nargs="+", type=int, help="Specific k values to try (default: all factors of L)")
    o = p.add_argument_group("output options")
    o.add_argument("--quiet", action="store_true", help="Minimal output")
    o.add_argument("--verbose", action="store_true", help="Verbose output including device and model summaries")
    o.add_argument("--save-solution", help="Save solution to JSON file")
    o.add_argument("--no-plot", action="store_true", help="Disable plotting of k vs objective curve")
    return p


def main(argv=None) -> int:
    parser = _parser()
    args = parser.parse_args(argv)
    bar = "=" * 60
    if args.profile:
        devices, model = load_from_profile_folder(args.profile)
        if not args.quiet:
            print(f"Loaded profile from: {args.profile}")
    elif args.devices and args.model:
        devices, model = load_devices_and_model(args.devices, args.model)
        if not args.quiet:
            print(f"Loaded {len(args.devices)} device file(s) and model")
    elif args.devices:
        parser.error("--devices requires --model")
    else:
        parser.error("Either --profile or both --devices and --model must be provided.")

    if args.verbose:
        print(f"\n{bar}\nLoaded {len(devices)} device(s):\n{bar}")
        for i, dev in enumerate(devices, 1):
            print(f"\n{i}. {dev.name}")
            dev.print_summary()
        model.print_summary()
    elif not args.quiet:
        print(f"\nLoaded {len(devices)} device(s) and model with {model.L} layers")

    if not args.quiet:
        print(f"\n{bar}\nRunning HALDA solver...\n{bar}")
    result = halda_solve(devices, model, mip_gap=args.mip_gap, plot=not args.no_plot, kv_bits="4bit")

    if args.quiet:
        print(f"k={result.k}, obj={result.obj_value:.6f}")
        for dev, wi in zip(devices, result.w):
            print(f"{dev.name}: {wi}")
    else:
        result.print_solution(devices)

    if args.save_solution:
        payload = {
            "k": result.k,
            "objective_value": result.obj_value,
            "layer_distribution": {d.name: {"w": wi, "n": ni} for d, wi, ni in zip(devices, result.w, result.n)},
            "sets": {name: [devices[i].name for i in idx] for name, idx in result.sets.items()},
        }
        with open(args.save_solution, "w") as f:
            json.dump(payload, f, indent=2)
        if not args.quiet:
            print(f"\nSolution saved to: {args.save_solution}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
