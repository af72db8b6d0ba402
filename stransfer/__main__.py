from styletransfer_amd.clis import cli

if __name__ == "__main__":
    cli(prog_name="stransfer")
