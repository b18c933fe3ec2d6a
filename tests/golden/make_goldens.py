"""Regenerate the committed fixtures under tests/golden/ from the reference.

Run in the build container only (the reference is not on the GPU box):
    python tests/golden/make_goldens.py [/root/reference]

Fixtures (all data, no reference source):
  archway_vertices.txt   copy of Radiance_Map_Data/vertices.txt: the GPU
                         engine's archway scene after loading (96 surfaces in
                         Surface(v1,v3,v2) order, then 6 lights), written by
                         Scene::save_vertices_to_file (GPU/scenes/scene.cu:63-88)
  triangle_o_pin.json    constants of Triangle::intersects read from the
                         prebuilt CPU object triangle.cpp.o (.rodata words the
                         function's relocations point at) and the order of its
                         accept tests, as disassembled
  cornell_ref_stats.json block means of Images/cornell/*.png (statistical
                         reference renders of the GPU engine, 720x720)
  scenes_ref_stats.json  block means of the OBJ scenes' reference renders, and of the
                         pretrained renderer's NN renders and the SARSA renders
  nn_ref_stats.json      the Neural-Q training logs of the shipped networks
  sarsa_ref_stats.json   the reference's Expected-SARSA training statistics
                         (Radiance_Map_Data/sarsa_*.txt, written per frame by
                         GPU/main.cu:321-339: average path length, 0.0,
                         zero-contribution light paths), per scene
"""
import json
import os
import re
import shutil
import struct
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def rodata_words(obj):
    out = subprocess.run(["objdump", "-s", "-j", ".rodata", obj], capture_output=True, text=True,
                         check=True).stdout
    data = bytearray()
    for line in out.splitlines():
        m = re.match(r"^\s*([0-9a-f]{4,})\s+((?:[0-9a-f]{1,8}\s?){1,4})", line)
        if m:
            data += bytes.fromhex("".join(m.group(2).split()))
    return bytes(data)


def main(ref):
    shutil.copy(os.path.join(ref, "Radiance_Map_Data", "vertices.txt"),
                os.path.join(HERE, "archway_vertices.txt"))

    obj = os.path.join(ref, "Old_CPU_Rendering_Engine", "CMakeFiles", "Monte_Carlo_Raytracer.dir",
                       "Source", "objects", "triangle.cpp.o")
    ro = rodata_words(obj)
    # relocations of Triangle::intersects: .rodata+0x20 (D scale), +0x14 (1.0), +0x24 (eps);
    # R_X86_64_PC32 addend -4 convention -> the word at addend+4
    word = lambda off: struct.unpack_from("<I", ro, off)[0]
    pin = {
        "t_scale_word": hex(word(0x24)),        # 512.0f = SCREEN_HEIGHT
        "one_word": hex(word(0x18)),            # 1.0f (u + v <= 1)
        "eps_word": hex(word(0x28)),            # 1e-5f
        "accept_order": ["detA != 0", "t >= 0", "u >= 0", "v >= 0", "u + v <= 1",
                         "t < dist + eps", "t > eps"],
        "solve": "inv = 1/detA; t = det_t*inv; u = det_u*inv; v = det_v*inv",
        "determinant": "((m00*(m11*m22 - m21*m12)) - m10*(m01*m22 - m21*m02)) + m20*(m01*m12 - m11*m02)",
    }
    with open(os.path.join(HERE, "triangle_o_pin.json"), "w") as f:
        json.dump(pin, f, indent=1)

    sarsa = {}
    for scene, fname in (("door_room", "sarsa_door_scene.txt"), ("archway", "sarsa_archway.txt"),
                         ("cornell", "sarsa_cornell.txt"),
                         ("complex_light_room", "sarsa_complex_light_scene.txt")):
        rows = [line.split() for line in open(os.path.join(ref, "Radiance_Map_Data", fname)) if line.strip()]
        sarsa[scene] = {"avg_path_length": [float(r[0]) for r in rows],
                        "zero_contribution_paths": [int(float(r[2])) for r in rows]}
    sarsa["_note"] = ("GPU engine, SCREEN 720x720 (constants/image_settings.h) and SAMPLES_PER_PIXEL 32 "
                      "(constants/monte_carlo_settings.h) at HEAD; the settings of the recorded runs are "
                      "not stated in the repository")
    with open(os.path.join(HERE, "sarsa_ref_stats.json"), "w") as f:
        json.dump(sarsa, f)

    try:
        import numpy as np
        from PIL import Image
        stats = {}
        for name in ("2048_2_default.png", "2048_300_default.png", "reference.png"):
            p = os.path.join(ref, "Images", "cornell", name)
            a = np.asarray(Image.open(p).convert("RGB"), np.float64)
            h, w, _ = a.shape
            b = 45  # 16x16 grid of 45x45 blocks
            blocks = a[: h // b * b, : w // b * b].reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))
            stats[name] = {"shape": [h, w], "block": b, "means": blocks.round(4).tolist()}
        with open(os.path.join(HERE, "cornell_ref_stats.json"), "w") as f:
            json.dump(stats, f)
    except ImportError:
        pass
    scene_image_stats(ref)
    nn_training_stats(ref)


def scene_image_stats(ref):
    """scenes_ref_stats.json: 45x45 block means of the reference renders of the OBJ scenes
    (Images/<scene>/reference.png, GPU engine, 720x720)."""
    try:
        import numpy as np
        from PIL import Image
    except ImportError:
        return
    stats = {}
    # (key, file): the 4096-spp reference of each scene, and the door room's 128-spp
    # default render (the thesis's comparison renders of that room were made of this scene;
    # its reference.png was made with other settings)
    files = [(s, f"Images/{s}/reference.png") for s in ("door_room", "archway", "complex_light")]
    files += [("door_room_default_128spp", "Images/door_room/default_128spp_50avg.png"),
              ("door_room_sarsa_128spp", "Images/door_room/sarsa_128_spp_avg_pl_5_max_pl_80.png"),
              # the pretrained renderer's own renders (PretrainedPathtracer, 128 spp) with the
              # networks Radiance_Map_Data/door_room_12_12.model and cornell_12_12.model
              ("door_room_nn_128spp", "Images/door_room/nn_128spp_32avg.png"),
              ("cornell_nn_128spp", "Images/cornell/nn_128spp_avg.png"),
              ("cornell_default_128spp", "Images/cornell/default_128spp_6avg.png"),
              # Expected-SARSA renders of the other scenes (128 spp)
              ("cornell_sarsa_128spp", "Images/cornell/sarsa_128spp_3avg_44Mb.png"),
              ("archway_sarsa_128spp", "Images/archway/sarsa_128spp_3avg_272Mb.png"),
              ("complex_light_sarsa_128spp", "Images/complex_light/sarsa_128spp_5avg_300Mb.png"),
              ("archway_default_128spp", "Images/archway/default_128spp_60avg.png"),
              ("complex_light_default_128spp", "Images/complex_light/default_128spp_58avg.png")]
    for key, rel in files:
        p = os.path.join(ref, rel)
        if not os.path.exists(p):
            continue
        a = np.asarray(Image.open(p).convert("RGB"), np.float64)
        h, w, _ = a.shape
        b = 45
        blocks = a[: h // b * b, : w // b * b].reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))
        stats[key] = {"file": rel, "shape": [h, w], "block": b, "means": blocks.round(4).tolist()}
    with open(os.path.join(HERE, "scenes_ref_stats.json"), "w") as f:
        json.dump(stats, f)


def nn_training_stats(ref):
    """nn_ref_stats.json: the Neural-Q training logs that produced the shipped networks
    (Radiance_Map_Data/*_stats*.txt / cornell_no_decay.txt, one line per training frame written by
    NeuralQPathtracer: average path length, loss, zero-contribution paths): all rows and the mean
    of the last 10."""
    out = {}
    for key, fname, model in (("door_room_12_12", "door_room_12_12_stats.txt", "door_room_12_12.model"),
                              ("cornell_12_12", "cornell_stats_12_12.txt", "cornell_12_12.model"),
                              ("cornell_no_decay", "cornell_no_decay.txt", "cornell_no_decay.model"),
                              # (runs whose networks the reference does not ship)
                              ("archway_12_12", "archway_12_12.txt", None),
                              ("complex_light_room_12_12", "complex_light_room_12_12.txt", None),
                              ("nn_training_stats", "nn_training_stats.txt", None)):
        rows = [[float(x) for x in line.split()] for line in open(os.path.join(ref, "Radiance_Map_Data", fname))
                if line.strip()]
        tail = rows[-10:]
        out[key] = {"file": "Radiance_Map_Data/" + fname, "model": model and "Radiance_Map_Data/" + model,
                    "avg_path_length": [r[0] for r in rows], "loss": [r[1] for r in rows],
                    "zero_contribution_paths": [r[2] for r in rows],
                    "last10_mean_path_length": round(sum(r[0] for r in tail) / len(tail), 4)}
    with open(os.path.join(HERE, "nn_ref_stats.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
